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
