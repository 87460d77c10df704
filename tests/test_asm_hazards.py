"""Static checks on the compiled gfx950 assembly of the hand-written kernels (no GPU needed).

1. The weight-stationary Q/K/V and one-pass FFN1 kernels issue their MFMAs as asm statements
   (qtx_ws.h mfma_asm / mfma_pin), so the compiler inserts none of the wait states MFMA results
   need before other instructions touch them: k_gemm_wss once read accumulators 13-17 wait
   states after their MFMA (copies at its loop latch), 0.5-5 % of Q/K/V outputs wrong.
   tools/check_asm_mfma.py scans those kernels.
2. VM_CNT_ORDER (csrc/qtx_common.h): a hand-counted vmcnt(N) that waits for an LDS-DMA is
   exact only when the N youngest vector-memory operations are loads; tools/check_vmcnt_order.py
   checks every hand-written counted wait of every product source (the KP row GEMM's
   vmcnt(8) / vmcnt(10) rings included) and is itself checked on a kernel that breaks the rule.
3. The weight-stationary kernels store inside their block loops, so their waits are vmcnt(0)."""
import os
import re
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "onnx-transformer_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
         "--cuda-device-only", "-S"]
needs_hipcc = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")


def _asm(tmp_path, src, name, extra=()):
    out = tmp_path / (name + ".s")
    subprocess.run([HIPCC, *FLAGS, *extra, "-o", str(out), src], check=True, capture_output=True,
                   timeout=600)
    return str(out)


@needs_hipcc
def test_asm_mfma_wait_states(tmp_path):
    s = _asm(tmp_path, os.path.join(CSRC, "qtx_wsgemm.hip"), "ws")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools/check_asm_mfma.py"), s,
                        "k_gemm_wsq", "k_gemm_wsy"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    for k in ("k_gemm_wsq", "k_gemm_wsy"):
        assert f"{k}: 0 hazards" in r.stdout, r.stdout[-2000:]


@needs_hipcc
def test_asm_mfma_wait_states_diag(tmp_path):
    """The diagnostic build's asm-MFMA kernels, the 32x32x32 ones (16-pass results) included."""
    s = _asm(tmp_path, os.path.join(CSRC, "diag", "qtx_wsgemm_diag.hip"), "wsd", ["-DQTX_DIAG"])
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools/check_asm_mfma.py"), s,
                        "k_gemm_wsq32", "k_gemm_wsy32"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    for k in ("k_gemm_wsq32", "k_gemm_wsy32"):
        assert f"{k}: 0 hazards" in r.stdout, r.stdout[-2000:]


@needs_hipcc
@pytest.mark.parametrize("src", ["qtx_gemm.hip", "qtx_wsgemm.hip", "qtx_attn.hip", "qtx_decode.hip",
                                 "qtx_kernels.hip", "qtx_ffn.hip"])
def test_counted_vmcnt_waits_follow_dmas_only(tmp_path, src):
    s = _asm(tmp_path, os.path.join(CSRC, src), src.split(".")[0])
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools/check_vmcnt_order.py"), s],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    if src in ("qtx_gemm.hip", "qtx_ffn.hip"):   # the rings' counted waits are really checked
        n = int(re.search(r"(\d+) counted vmcnt waits", r.stdout).group(1))
        assert n > 0, r.stdout


@needs_hipcc
def test_vmcnt_checker_flags_a_store_behind_the_dma(tmp_path):
    """Negative control: a loop whose counted wait has a store among the youngest operations."""
    src = tmp_path / "bad.hip"
    src.write_text(r'''
#include <hip/hip_runtime.h>
__global__ void k_bad(const int* a, int* o, int n) {
  __shared__ int l[1024];
  for (int i = 0; i < n; ++i) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(l + 64 * (i & 3)));
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(a + i * 64 + threadIdx.x), "s"(dst) : "memory");
    o[i * 64 + threadIdx.x] = l[threadIdx.x];
    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  }
}
''')
    s = _asm(tmp_path, str(src), "bad")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools/check_vmcnt_order.py"), s],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "global_store" in r.stdout, r.stdout


def test_ws_kernels_wait_vmcnt_zero():
    """VM_CNT_ORDER in the source: the weight-stationary product kernels store inside their
    block loops, so their hand-written waits must be vmcnt(0) (the race fixed in round 3)."""
    src = open(os.path.join(CSRC, "qtx_wsgemm.hip")).read()
    code = "\n".join(l.split("//")[0] for l in src.splitlines())
    assert not re.search(r"WAIT_VM\(\s*[1-9]", code), "counted WAIT_VM in a ws kernel"
    assert not re.search(r"vmcnt\(\s*[1-9]", code), "counted vmcnt in a ws kernel"


def test_product_sources_read_no_environment_per_launch():
    """Product hygiene: kernels and launchers read their switches through qtx_knobs.h (once),
    never getenv() per launch; measured-negative variants live in csrc/diag/qtx_wsgemm_diag.hip, which
    only the diagnostic build compiles."""
    sys.path.insert(0, os.path.join(REPO, "onnx-transformer_amd"))
    from qtx import _build
    for f in _build.SOURCES:
        code = open(os.path.join(CSRC, f)).read()
        if f == "qtx_knobs.hip":
            continue
        assert "getenv(" not in code, f"{f} reads the environment outside qtx_knobs"
    assert not any("diag" in f for f in _build.SOURCES)
    assert all(f.startswith("diag/") for f in _build.DIAG_SOURCES)
