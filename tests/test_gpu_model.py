"""Module-level parity of the HIP path (through the C-ABI and the reference-shaped host
API) against the CPU oracle: encoder graph, decoder graph, greedy decode — bit-exact."""
import numpy as np
import pytest

from oracle import qtx_oracle as O

pytestmark = pytest.mark.gpu
f32 = np.float32


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def make_batch(rng, B, S, lens=None):
    src = np.full((B, S), 2, np.int64)
    lens = lens if lens is not None else rng.integers(4, S + 1, B)
    for b, n in enumerate(lens):
        src[b, 0] = 0
        src[b, 1:n - 1] = rng.integers(4, 5337, max(n - 2, 0))
        src[b, n - 1] = 1
    return src, (src != 2)[:, None, :]


def test_encoder_session_matches_oracle(torch, gpu_model, oracle_model, golden_model):
    from qtx.session import InferenceSession
    sess = InferenceSession("./onnx/fixed/encoder_fixed.onnx", model=gpu_model)
    feeds = {"global_in": golden_model["enc_in"], "global_in_1": golden_model["src_mask"]}
    (out,) = sess.run(None, feeds)
    ref = oracle_model.encode(golden_model["enc_in"], golden_model["src_mask"])
    np.testing.assert_array_equal(out, ref)


def test_decoder_run_module_matches_oracle(torch, gpu_model, oracle_model, golden_model):
    from qtx.session import run_module
    feeds = {"global_in": golden_model["dec_in"], "global_in_1": golden_model["memory"],
             "global_in_2": golden_model["src_mask"], "global_in_3": golden_model["tgt_mask"]}
    outs, wd = run_module("decoder", feeds, "./onnx/fixed/decoder_fixed.onnx", {}, None,
                          model=gpu_model)
    ref = oracle_model.decode(golden_model["dec_in"], golden_model["memory"],
                              golden_model["src_mask"], golden_model["tgt_mask"])
    np.testing.assert_array_equal(outs["global_out"], ref)
    assert wd["global_out"] is outs["global_out"] and "global_in_3" in wd


def test_encoder_larger_batch(torch, gpu_model, oracle_model):
    rng = np.random.default_rng(5)
    src, m = make_batch(rng, 5, 72)
    x = oracle_model.embed(src, oracle_model.src_lut)
    out = gpu_model.encode(torch.from_numpy(x).cuda(),
                           torch.from_numpy(m.reshape(5, 72).astype(np.uint8)).cuda())
    np.testing.assert_array_equal(out.cpu().numpy(), oracle_model.encode(x, m))


def test_greedy_decode_matches_oracle(torch, gpu_model, oracle_model, golden_model):
    from qtx.decode import greedy_decode
    ys = greedy_decode(gpu_model, golden_model["src"], golden_model["src_mask"], 72, 0)
    ref = oracle_model.greedy_decode(golden_model["src"], golden_model["src_mask"], 72)
    np.testing.assert_array_equal(ys, ref)


@pytest.mark.parametrize("env", [{"QTX_NO_GRAPH": "1"}, {"QTX_UNFUSED": "1"},
                                 {"QTX_GRAPH_STEPS": "13"}, {"QTX_DECODE_GROUPS": "3"},
                                 {"QTX_DECODE_GROUPS": "2", "QTX_NO_GRAPH": "1"},
                                 {"QTX_FFN_QKERNEL": "1"}])
def test_greedy_paths_agree(torch, gpu_model, knob_env, env):
    """The fused+graph decode step, the fused eager step, the unfused kernels, graphs of
    several steps and sub-batches on several streams agree."""
    from qtx.decode import greedy_decode
    src, m = make_batch(np.random.default_rng(5), 5, 24, lens=[24, 20, 9, 17, 3])
    ref = greedy_decode(gpu_model, src, m, 40, 0)
    for k, v in env.items():
        knob_env(k, v)
    np.testing.assert_array_equal(greedy_decode(gpu_model, src, m, 40, 0), ref)


@pytest.mark.diag
@pytest.mark.parametrize("env", [{"QTX_DECODE_GROUPS": "2", "QTX_GROUP_GRAPH": "1"},
                                 {"QTX_SPLIT_LN": "1"}, {"QTX_DEVICE_STEP": "1"},
                                 {"QTX_ATTN_PMAX": "1"}, {"QTX_FFN_PMAX": "1"},
                                 {"QTX_HQUANT_ROWS": "1"}])
def test_greedy_diag_paths_agree(torch, gpu_model, knob_env, env):
    """The measured-negative decode alternatives of the diagnostic build (csrc/qtx_knobs.h
    QTX_DKNOB: one graph with sub-batch branches, separate LayerNorm kernels, the device
    position counter, per-head / per-tile partial maxima, the hidden quantized by k_rows)
    give the product step's ids."""
    test_greedy_paths_agree(torch, gpu_model, knob_env, env)


def test_greedy_default_groups_at_512(torch, gpu_model, knob_env):
    """From B = 512 the decode runs as two sub-batch graphs on two streams by default
    (qtx_api.hip decode_groups); its ids equal the one-graph decode's."""
    from qtx.decode import greedy_decode
    rng = np.random.default_rng(12)
    src, m = make_batch(rng, 512, 24, lens=list(rng.integers(3, 25, 512)))
    two = greedy_decode(gpu_model, src, m, 24, 0)
    knob_env("QTX_DECODE_GROUPS", 1)
    np.testing.assert_array_equal(greedy_decode(gpu_model, src, m, 24, 0), two)


def test_greedy_long_source_unfused_path(torch, gpu_model, oracle_model):
    """Sources longer than the fused kernel's 128-key LDS budget take the unfused path."""
    from qtx.decode import greedy_decode
    rng = np.random.default_rng(9)
    src, m = make_batch(rng, 2, 160, lens=[160, 100])
    ys = greedy_decode(gpu_model, src, m, 10, 0)
    np.testing.assert_array_equal(ys, oracle_model.greedy_decode(src, m, 10))


def test_greedy_batch_invariance(torch, gpu_model):
    """Per-token quantization makes results batch-composition invariant:
    a sentence decoded inside a batch of 32 equals it decoded alone."""
    from qtx.decode import greedy_decode
    rng = np.random.default_rng(11)
    src, m = make_batch(rng, 32, 72)
    ys = greedy_decode(gpu_model, src, m, 72, 0)
    for b in (0, 17, 31):
        one = greedy_decode(gpu_model, src[b:b + 1], m[b:b + 1], 72, 0)
        np.testing.assert_array_equal(one[0], ys[b])
    assert (ys[:, 0] == 0).all() and ys.min() >= 0 and ys.max() < 4444


def test_feed_validation(torch, gpu_model, golden_model):
    from qtx.session import InferenceSession
    sess = InferenceSession("encoder", model=gpu_model)
    with pytest.raises(ValueError, match="missing"):
        sess.run(None, {"global_in": golden_model["enc_in"]})
    with pytest.raises(ValueError):
        sess.run(None, {"global_in": golden_model["enc_in"][..., :256],
                        "global_in_1": golden_model["src_mask"]})


def test_int4_model_matches_oracle(torch, state_dict, golden_model):
    from qtx.model import QtxModel
    from qtx.weights import ModelConfig
    m4 = QtxModel(state_dict, ModelConfig(weight_bits=4))
    o4 = O.OracleModel(state_dict, n_bits=4)
    x, mk = golden_model["enc_in"], golden_model["src_mask"]
    out = m4.encode(torch.from_numpy(x).cuda(),
                    torch.from_numpy(mk.reshape(2, -1).astype(np.uint8)).cuda())
    np.testing.assert_array_equal(out.cpu().numpy(), o4.encode(x, mk))
    from qtx.decode import greedy_decode
    ys = greedy_decode(m4, golden_model["src"], golden_model["src_mask"], 24, 0)
    np.testing.assert_array_equal(ys, o4.greedy_decode(golden_model["src"],
                                                       golden_model["src_mask"], 24))


@pytest.mark.parametrize("B,S,max_len", [(3, 13, 23), (2, 9, 18), (5, 31, 37)])
def test_greedy_ragged_groups_matches_oracle(torch, gpu_model, oracle_model, B, S, max_len):
    """Source lengths and max_len that are not multiples of 4: the decode's value caches
    are kept in 4-key groups (k_dec_attn, k_vgroup4; padded last group), so the self cache's
    last group is partial every step and the cross values' last group is zero-padded."""
    from qtx.decode import greedy_decode
    rng = np.random.default_rng(B * 100 + S)
    src, m = make_batch(rng, B, S)
    ys = greedy_decode(gpu_model, src, m, max_len, 0)
    np.testing.assert_array_equal(ys, oracle_model.greedy_decode(src, m, max_len))
