"""The BASELINE configurations the bench measures, at their full sizes, under test.

* cfg3 — encoder forward at B=256, S=128.  A batch of >= 256 sentences takes the
  two-stream sub-batch path (csrc/qtx_api.hip, enc_split: fork / lag / join events); it
  must equal the single-stream path (QTX_ENC_NOSPLIT=1), the same sentences encoded in
  batches of 8 (other kernels: k_attn_mfma instead of k_attn_encq, partial row tiles)
  and, on sampled sentences, the CPU oracle — all bit for bit.  Two threads sharing the
  model handle run the split path concurrently (the shared events).
* cfg5 — the per-GPU shard of the 8-GPU config: greedy decode of 256 sentences, equal to
  the same sentences decoded as 8 batches of 32 and, on a sample, to the oracle.
* cfg4 — int4 weights, greedy decode at B=32, against OracleModel(n_bits=4) on a sample.

Oracle samples are small (the numpy oracle takes seconds per sentence); the full-size
checks are the size-independent properties above (batch-composition invariance, path
agreement), which hold because every quantizer is per token.
"""
import threading

import numpy as np
import pytest

from oracle import qtx_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def make_src(rng, B, S, lens):
    src = np.full((B, S), 2, np.int64)
    for b, n in enumerate(lens):
        src[b, 0] = 0
        src[b, 1:n - 1] = rng.integers(4, 5337, max(n - 2, 0))
        src[b, n - 1] = 1
    return src, (src != 2)[:, None, :]


@pytest.fixture(scope="module")
def cfg3_inputs(oracle_model):
    """256 sentences of 128 tokens (cfg3 is full length; every 16th sentence is padded
    so the key mask is exercised too)."""
    rng = np.random.default_rng(303)
    lens = np.full(256, 128)
    lens[::16] = rng.integers(9, 128, 16)
    src, m = make_src(rng, 256, 128, lens)
    x = oracle_model.embed(src, oracle_model.src_lut)
    return x, m


def _encode(torch, model, x, m):
    B, S = m.shape[0], m.shape[-1]
    out = model.encode(torch.from_numpy(x).cuda(),
                       torch.from_numpy(m.reshape(B, S).astype(np.uint8)).cuda())
    return out.cpu().numpy()


@pytest.fixture(scope="module")
def cfg3_split(torch, gpu_model, cfg3_inputs):
    x, m = cfg3_inputs
    return _encode(torch, gpu_model, x, m)


@pytest.mark.parametrize("env", [pytest.param({"QTX_FFN_FUSED_MIN_M": 1}, marks=pytest.mark.diag),
                                 {"QTX_NO_WSX": 1}])
def test_cfg3_encoder_ffn_paths_agree(torch, gpu_model, cfg3_inputs, cfg3_split, knob_env, env):
    """The default encoder (the one-pass FFN1 with the in-launch exchange + the FFN2 row
    GEMM) against the fused FFN launch (k_ffn_fused, QTX_FFN_FUSED_MIN_M: diagnostic build) and the two-pass
    FFN1 (QTX_NO_WSX), which also runs the batch as two half-batch streams — the same bits."""
    x, m = cfg3_inputs
    for k, v in env.items():
        knob_env(k, v)
    np.testing.assert_array_equal(_encode(torch, gpu_model, x, m), cfg3_split)


def test_cfg3_encoder_equals_batches_of_8(torch, gpu_model, cfg3_inputs, cfg3_split):
    x, m = cfg3_inputs
    for b0 in range(0, 256, 8):
        np.testing.assert_array_equal(_encode(torch, gpu_model, x[b0:b0 + 8], m[b0:b0 + 8]),
                                      cfg3_split[b0:b0 + 8], err_msg=f"sentences {b0}..{b0 + 7}")


@pytest.mark.parametrize("b", [0, 5, 37, 64, 127, 128, 191, 200, 254, 255])
def test_cfg3_encoder_sample_matches_oracle(torch, oracle_model, cfg3_inputs, cfg3_split, b):
    """Ten of the 256 sentences against the oracle, bit for bit: 0-127 sit in the first half
    of the two-stream split, 128-255 in the second; the first and last row blocks of each
    half (0, 127, 128, 255), padded sentences (0, 64, 128), and rows that the one-pass FFN1's
    row groups put on different XCDs.  The other 246 are pinned through the batch-invariance
    and path-agreement tests above."""
    x, m = cfg3_inputs
    np.testing.assert_array_equal(cfg3_split[b:b + 1], oracle_model.encode(x[b:b + 1], m[b:b + 1]))


@pytest.mark.parametrize("env", [{}, pytest.param({"QTX_FFN_FUSED_MIN_M": 1}, marks=pytest.mark.diag)])
def test_cfg3_encoder_split_two_threads(torch, gpu_model, cfg3_inputs, cfg3_split, knob_env, env):
    """Two threads share the model handle, each on its own stream with its own inputs, at
    the same time, with the one-pass FFN1 whose workgroups wait for their partner slices
    (work by arrival ticket: no co-residency requirement; the default) and with the fused
    FFN launch.
    One round each: the ordering rule these launches depend on (a counted vmcnt never waits
    past a store, qtx_common.h VM_CNT_ORDER) is checked statically on every CPU run
    (tests/test_asm_hazards.py), not by repetition here."""
    for k, v in env.items():
        knob_env(k, v)
    x, m = cfg3_inputs
    x2 = np.ascontiguousarray(x[::-1])      # a different batch: the sentences reversed
    m2 = np.ascontiguousarray(m[::-1])
    _two_threads_round(torch, gpu_model, x, m, x2, m2, cfg3_split)


def _two_threads_round(torch, gpu_model, x, m, x2, m2, cfg3_split):
    res, errs = {}, []

    def run(tag, xx, mm):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                xd = torch.from_numpy(xx).cuda()
                md = torch.from_numpy(mm.reshape(256, 128).astype(np.uint8)).cuda()
                outs = [gpu_model.encode(xd, md) for _ in range(3)]
                s.synchronize()
            res[tag] = [o.cpu().numpy() for o in outs]
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=run, args=("a", x, m)),
          threading.Thread(target=run, args=("b", x2, m2))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for o in res["a"]:
        np.testing.assert_array_equal(o, cfg3_split)
    for o in res["b"]:
        np.testing.assert_array_equal(o, cfg3_split[::-1])


def _cfg2_src(seed, B):
    """src <= 64 tokens padded to 72 (BASELINE configs 2 / 5)."""
    rng = np.random.default_rng(seed)
    return make_src(rng, B, 72, rng.integers(8, 65, B))


def test_cfg5_greedy_256_equals_batches_of_32(torch, gpu_model, oracle_model):
    from qtx.decode import greedy_decode
    src, m = _cfg2_src(505, 256)
    ys = greedy_decode(gpu_model, src, m, 72, 0)
    assert ys.shape == (256, 72) and (ys[:, 0] == 0).all()
    for b0 in range(0, 256, 32):
        np.testing.assert_array_equal(greedy_decode(gpu_model, src[b0:b0 + 32], m[b0:b0 + 32], 72, 0),
                                      ys[b0:b0 + 32], err_msg=f"sentences {b0}..{b0 + 31}")
    for b in (77, 250):
        np.testing.assert_array_equal(ys[b:b + 1],
                                      oracle_model.greedy_decode(src[b:b + 1], m[b:b + 1], 72))


def test_cfg4_int4_greedy_b32_matches_oracle(torch, state_dict):
    """The 4-bit model's decode (its weights unpacked to int8 for the step kernels) equals
    the oracle on a sample."""
    from qtx.decode import greedy_decode
    from qtx.model import QtxModel
    from qtx.weights import ModelConfig
    m4 = QtxModel(state_dict, ModelConfig(weight_bits=4))
    src, m = _cfg2_src(404, 32)
    ys = greedy_decode(m4, src, m, 72, 0)
    o4 = O.OracleModel(state_dict, n_bits=4)
    pick = np.array([0, 9, 20, 31])
    np.testing.assert_array_equal(ys[pick], o4.greedy_decode(src[pick], m[pick], 72))
    # the int4 model is a different model: its tokens differ from the int8 ones
    ys8 = greedy_decode(QtxModel(state_dict), src[:4], m[:4], 72, 0)
    assert (ys8 != ys[:4]).any()


@pytest.mark.diag
def test_cfg4_int4_packed_step_same_ids(torch, state_dict, knob_env):
    """The diagnostic build's decode step on the packed int4 kernels (QTX_INT4_PACKED,
    measured 5.7 % slower) gives the unpacked step's ids for the whole batch."""
    from qtx.decode import greedy_decode
    from qtx.model import QtxModel
    from qtx.weights import ModelConfig
    m4 = QtxModel(state_dict, ModelConfig(weight_bits=4))
    src, m = _cfg2_src(404, 32)
    ys = greedy_decode(m4, src, m, 72, 0)
    knob_env("QTX_INT4_PACKED", 1)
    np.testing.assert_array_equal(greedy_decode(m4, src, m, 72, 0), ys)


def test_greedy_fresh_buffers_reuse_graph(torch, gpu_model):
    """Fresh id / mask tensors per call (the public greedy_decode path) give the same ids
    as the bench's reused buffers (the graph cache no longer keys on them)."""
    src, m = _cfg2_src(606, 32)
    srcd = torch.from_numpy(src).cuda()
    md = torch.from_numpy(m.reshape(32, 72).astype(np.uint8)).cuda()
    out = torch.empty((32, 72), dtype=torch.int64, device="cuda")
    gpu_model.greedy(srcd, md, 72, 0, out=out)
    ref = out.cpu().numpy()
    for _ in range(3):
        ids = gpu_model.greedy(srcd.clone(), md.clone(), 72, 0)
        np.testing.assert_array_equal(ids.cpu().numpy(), ref)
