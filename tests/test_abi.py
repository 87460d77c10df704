"""The C-ABI library builds, loads without a GPU and exports every symbol of include/qtx.h."""
import ctypes

from qtx import _build, _lib


def test_library_builds_and_loads():
    path = _build.build()
    L = ctypes.CDLL(path)
    assert L is not None
    assert _lib.lib().qtx_version().decode().startswith("qtx")


def test_every_header_symbol_exported():
    names = _lib.header_symbols()
    assert len(names) >= 18
    L = ctypes.CDLL(_build.LIB)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # the ctypes signature table covers the whole header, and nothing else
    assert sorted(_lib.SIGNATURES) == names


def test_tensor_count_matches_host_order():
    from qtx.weights import ModelConfig, tensor_order
    for cfg in (ModelConfig(), ModelConfig(n_layers=2), ModelConfig(weight_bits=4)):
        c = _lib.QtxConfig(cfg.src_vocab, cfg.tgt_vocab, cfg.n_layers, cfg.d_model, cfg.d_ff,
                           cfg.n_heads, cfg.max_len, cfg.weight_bits)
        assert _lib.lib().qtx_model_tensor_count(ctypes.byref(c)) == len(tensor_order(cfg))


def test_invalid_config_rejected_without_gpu():
    c = _lib.QtxConfig(5337, 4444, 6, 384, 2048, 6, 5000, 8)   # d_model 384 unsupported
    assert _lib.lib().qtx_model_tensor_count(ctypes.byref(c)) == -1
    assert b"d_model" in _lib.lib().qtx_last_error()
    c = _lib.QtxConfig(5337, 4444, 6, 512, 2048, 8, 5000, 3)   # 3-bit weights
    h = ctypes.c_void_p()
    arr = (ctypes.c_void_p * 1)()
    rc = _lib.lib().qtx_model_create(ctypes.byref(c), arr, 1, None, None, ctypes.byref(h))
    assert rc != 0 and not h.value


def test_workspace_queries_without_model_are_zero():
    L = _lib.lib()
    assert L.qtx_encoder_workspace_size(None, 2, 16) == 0
    assert L.qtx_greedy_workspace_size(None, 2, 16, 72) == 0
