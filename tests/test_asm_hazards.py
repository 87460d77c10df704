"""The weight-stationary Q/K/V and one-pass FFN1 kernels issue their MFMAs as asm statements (qtx_wsgemm.hip
mfma_asm / mfma_pin), so the compiler inserts none of the wait states MFMA results need
before other instructions touch them: k_gemm_wss once read accumulators 13-17 wait states
after their MFMA (copies at its loop latch), 0.5-5 % of Q/K/V outputs wrong.  Compiles the
file to gfx950 assembly here (no GPU) and runs tools/check_asm_mfma.py on those kernels."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_asm_mfma_wait_states(tmp_path):
    src = os.path.join(REPO, "onnx-transformer_amd/csrc/qtx_wsgemm.hip")
    out = tmp_path / "ws.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-fast-math", "--cuda-device-only", "-S", "-o", str(out), src],
                   check=True, capture_output=True, timeout=600)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools/check_asm_mfma.py"), str(out),
                        "k_gemm_wsq", "k_gemm_wss", "k_gemm_wsy"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    for k in ("k_gemm_wsq", "k_gemm_wss", "k_gemm_wsy"):
        assert f"{k}: 0 hazards" in r.stdout, r.stdout[-2000:]


def test_ws_kernels_wait_vmcnt_zero():
    """VM_CNT_ORDER (csrc/qtx_common.h): the weight-stationary kernels store inside their
    block loops, and a store may retire before an LDS-DMA issued ahead of it, so their
    hand-written waits must be vmcnt(0) — a count that leaves stores in flight can release
    a barrier before the block's DMA landed (the race fixed in round 3)."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "onnx-transformer_amd", "csrc", "qtx_wsgemm.hip")).read()
    code = "\n".join(l.split("//")[0] for l in src.splitlines())
    assert not re.search(r"WAIT_VM\(\s*[1-9]", code), "counted WAIT_VM in a ws kernel"
    assert not re.search(r"vmcnt\(\s*[1-9]", code), "counted vmcnt in a ws kernel"
