"""The diagnostic build (csrc/diag/, libqtx_diag.so: the measured-negative kernel variants
of DESIGN.md §4 and the diagnostic switches) is kept compiling and bit-exact:
the CPU suite cross-compiles its sources for gfx950, the GPU suite runs every variant
against the oracle through the diagnostic library (tests/diag_variants.py, a subprocess:
one process loads one library)."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "onnx-transformer_amd", "csrc")
DIAG_LIB = os.path.join(REPO, "onnx-transformer_amd", "qtx", "libqtx_diag.so")


def test_diag_sources_compile(tmp_path):
    sys.path.insert(0, os.path.join(REPO, "onnx-transformer_amd"))
    from qtx import _build
    if not (shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc")):
        pytest.skip("no hipcc")
    flags = [f for f in _build.FLAGS if f != "-shared"] + ["-DQTX_DIAG"]
    for src in _build.DIAG_SOURCES:
        r = subprocess.run([_build.hipcc(), *flags, "-c", "-o", str(tmp_path / "d.o"),
                            os.path.join(CSRC, src)], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.gpu
def test_diag_variants_bit_exact():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(DIAG_LIB):          # normally prebuilt by __graft_entry__.build()
        sys.path.insert(0, os.path.join(REPO, "onnx-transformer_amd"))
        from qtx import _build
        _build.build(extra=["-DQTX_DIAG"])
    env = dict(os.environ, QTX_LIB_PATH=DIAG_LIB)
    r = subprocess.run([sys.executable, "-u", os.path.join(REPO, "tests", "diag_variants.py")],
                       capture_output=True, text=True, env=env, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.gpu
def test_diag_switch_paths():
    """The tests that force a diagnostic switch (marker diag: the measured-negative decode
    and GEMM alternatives of csrc/qtx_knobs.h QTX_DKNOB, constants in libqtx.so) run in one
    subprocess against libqtx_diag.so, where the switches are read."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(DIAG_LIB):
        sys.path.insert(0, os.path.join(REPO, "onnx-transformer_amd"))
        from qtx import _build
        _build.build(extra=["-DQTX_DIAG"])
    env = dict(os.environ, QTX_LIB_PATH=DIAG_LIB)
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", os.path.join(REPO, "tests"), "-q",
                        "-m", "gpu and diag", "-p", "no:cacheprovider", "--timeout", "120",
                        "--timeout-method", "thread"],
                       capture_output=True, text=True, env=env, timeout=600, cwd=REPO)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout and " skipped" not in r.stdout.splitlines()[-1], r.stdout[-500:]
