import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "onnx-transformer_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm gfx950 GPU (MI355X)")
    config.addinivalue_line("markers", "diag: forces a diagnostic switch (csrc/qtx_knobs.h "
                            "QTX_DKNOB): runs only against libqtx_diag.so, in the subprocess "
                            "of tests/test_diag_build.py::test_diag_switch_paths")


def _diag_lib():
    return "diag" in os.path.basename(os.environ.get("QTX_LIB_PATH", ""))


def pytest_collection_modifyitems(config, items):
    """The product library reads no diagnostic switch (they are constants there), so a test
    that forces one would silently run the default path: such tests (marker diag) run only
    in the process test_diag_build.py starts with QTX_LIB_PATH = libqtx_diag.so."""
    if _diag_lib():
        return
    skip = pytest.mark.skip(reason="diag switch: run against libqtx_diag.so by "
                                   "tests/test_diag_build.py::test_diag_switch_paths")
    for it in items:
        if "diag" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden_ops():
    return dict(np.load(os.path.join(GOLDEN, "golden_ops.npz")))


@pytest.fixture(scope="session")
def golden_model():
    return dict(np.load(os.path.join(GOLDEN, "golden_model.npz")))


@pytest.fixture(scope="session")
def state_dict():
    from qtx.weights import synthetic_state_dict
    return synthetic_state_dict(20241223, ln_random=True)


@pytest.fixture(scope="session")
def oracle_model(state_dict):
    from oracle.qtx_oracle import OracleModel
    return OracleModel(state_dict)


@pytest.fixture(scope="session")
def gpu_model(state_dict):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from qtx.model import QtxModel
    return QtxModel(state_dict)


@pytest.fixture
def knob_env(monkeypatch):
    """Set library switches (csrc/qtx_knobs.h, read once per process) for one test: sets the
    variable and re-reads the switches; restores both at teardown."""
    from qtx import _lib

    def set_(name, value):
        monkeypatch.setenv(name, str(value))
        _lib.reload_knobs()
    yield set_
    monkeypatch.undo()
    _lib.reload_knobs()
