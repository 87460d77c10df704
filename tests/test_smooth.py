"""SmoothQuant fold (get_quantized_model.py:9-36,46-148): opt-in, bit-identical
to the reference's smooth_lm on the same weights, and off by default (the reference's
exported path reloads its checkpoint after smoothing, output.py:609-613)."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def scales():
    from qtx.weights import load_act_scales
    return load_act_scales(os.path.join(GOLDEN, "transformer_scales.npz"))


@pytest.fixture(scope="module")
def smoothed(state_dict, scales):
    from qtx.weights import smooth_state_dict
    return smooth_state_dict(state_dict, scales)


def test_fold_matches_reference_smooth_lm(state_dict, smoothed):
    g = dict(np.load(os.path.join(GOLDEN, "smooth_golden.npz")))
    changed = sorted(k[:-4] for k in g if k.endswith("|sum"))
    assert len(changed) == 126                  # 6 x 8 encoder + 6 x 13 decoder tensors
    for k in changed:
        v = np.asarray(smoothed[k], np.float32).ravel()
        idx = np.linspace(0, v.size - 1, 257).astype(np.int64)
        np.testing.assert_array_equal(v[idx], g[k + "|sample"], err_msg=k)
        assert np.float64(v.astype(np.float64).sum()) == pytest.approx(float(g[k + "|sum"]), rel=1e-12, abs=1e-9), k
    # and nothing else changed
    for k, v in state_dict.items():
        if k not in changed:
            assert smoothed[k] is v or np.array_equal(smoothed[k], v), k


def test_default_load_applies_nothing(tmp_path, state_dict, scales):
    import torch
    from qtx.weights import load_checkpoint
    p = str(tmp_path / "ck.pt")
    torch.save({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in state_dict.items()}, p)
    sd = load_checkpoint(p)
    for k, v in state_dict.items():
        np.testing.assert_array_equal(sd[k], v, err_msg=k)
    sm = load_checkpoint(p, smooth_scales=os.path.join(GOLDEN, "transformer_scales.npz"))
    assert not np.array_equal(sm["encoder.layers.0.sublayer.0.norm.a_2"],
                              state_dict["encoder.layers.0.sublayer.0.norm.a_2"])


def test_fold_keeps_float_function_of_first_block(state_dict, smoothed):
    """Before quantization the fold is an identity of the fp32 function LN -> Linear
    (a_2/s * xhat + b_2/s, then W * s): check on the encoder layer-0 QKV input."""
    from oracle import qtx_oracle as O
    x = np.random.default_rng(0).standard_normal((8, 512)).astype(np.float32)
    p = "encoder.layers.0"
    y0 = O.layer_norm(x, state_dict[f"{p}.sublayer.0.norm.a_2"], state_dict[f"{p}.sublayer.0.norm.b_2"])
    y1 = O.layer_norm(x, smoothed[f"{p}.sublayer.0.norm.a_2"], smoothed[f"{p}.sublayer.0.norm.b_2"])
    w0 = state_dict[f"{p}.self_attn.linears.0.weight"]
    w1 = smoothed[f"{p}.self_attn.linears.0.weight"]
    np.testing.assert_allclose(y1 @ w1.T, y0 @ w0.T, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_gpu_smoothed_model_matches_oracle(smoothed):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.qtx_oracle import OracleModel
    from qtx.decode import greedy_decode, make_src_mask
    from qtx.model import QtxModel
    rng = np.random.default_rng(5)
    src = np.full((3, 16), 2, np.int64)
    for b, n in enumerate([16, 11, 8]):
        src[b, 0], src[b, n - 1] = 0, 1
        src[b, 1:n - 1] = rng.integers(4, 5337, n - 2)
    mask = make_src_mask(src)
    ys = greedy_decode(QtxModel(smoothed), src, mask, 20, 0)
    ref = OracleModel(smoothed).greedy_decode(src, mask, 20)
    np.testing.assert_array_equal(ys, ref)
