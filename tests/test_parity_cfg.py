"""Quantitative reference parity at the BASELINE shapes (cfg3 encoder S=128, cfg2 S=72 with
the decoder teacher-forced over T=71), from fixtures the reference itself generated
(tests/golden/make_parity_cfg.py -> golden_parity_cfg.npz).

test_parity_quant.py replays the reference's rounding decisions layer by layer on 2 short
sentences; here the oracle runs each stack end to end (its own embedding, 6 layers, the
final norm) while taking the reference's decision at every activation quantizer
(quant_linear.py:30-43) and P quantization (attention.py:33-35), in call order, after
checking each differing code is one step at a near-tie of its own quotient
(replay_codes.Codes).  With those few hundred decisions replayed, every layer output
equals the reference's within fp32 noise (NOISE_REL; measured <= 5.4e-7), so every other
difference between the two is one of them.  The GPU path equals the oracle bit for bit
(tests/test_gpu_*.py), so this is the GPU path's parity too.
"""
import os
import sys

import numpy as np
import pytest

from oracle import qtx_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from replay_codes import Codes, decoder_chain, encoder_chain, sample_rows  # noqa: E402

f32 = np.float32
NOISE_REL = 2e-6


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(os.path.join(HERE, "golden", "golden_parity_cfg.npz")))


def _check_pass(fx, name, outs, codes):
    ref = fx[f"{name}_layers"]
    assert codes.i == codes.n_calls
    assert len(outs) == ref.shape[0]
    devs = [float(np.abs(sample_rows(a) - b).max() / np.abs(b).max()) for a, b in zip(outs, ref)]
    print(f"{name}: {codes.i} calls, {sum(codes.flips)} flips at {sum(codes.ties)} near-ties, "
          f"per-layer rel dev {['%.1e' % d for d in devs]}")
    assert devs[0] < 1e-6                       # the embedding: no quantizer upstream
    assert max(devs) < NOISE_REL
    return devs


@pytest.fixture(scope="module")
def enc2(fx, oracle_model):
    codes = Codes(sparse=Codes.unpack(fx, "enc2"))
    outs = encoder_chain(oracle_model, fx["src2"], fx["src_mask2"], codes)
    return outs, codes


def test_cfg3_encoder_replay(fx, oracle_model):
    """cfg3: 4 sentences x S = 128 (lengths 100..128), the encoder end to end."""
    codes = Codes(sparse=Codes.unpack(fx, "enc3"))
    outs = encoder_chain(oracle_model, fx["src3"], fx["src_mask3"], codes)
    _check_pass(fx, "enc3", outs, codes)
    assert sum(codes.flips) < 1e-3 * sum(int(s) for s in fx["enc3_size"])


def test_cfg2_encoder_replay(fx, enc2):
    _check_pass(fx, "enc2", *enc2)


def test_cfg2_decoder_replay(fx, oracle_model, enc2):
    """cfg2: the decoder teacher-forced over the reference's whole greedy prefix (8 x T = 71),
    on the oracle's replayed memory."""
    ys = fx["greedy2"][:, :71]
    codes = Codes(sparse=Codes.unpack(fx, "dec2"))
    outs = decoder_chain(oracle_model, ys, enc2[0][-1], fx["src_mask2"], codes)
    _check_pass(fx, "dec2", outs, codes)


def test_cfg2_replay_detects_a_changed_oracle(fx, oracle_model):
    """The CRC makes the sparse fixture a full one: an oracle whose codes moved by a step
    away from a tie is refused, not taken for the reference's."""
    codes = Codes(sparse=Codes.unpack(fx, "enc2"))
    real = O.quant_rows

    def off_by_one(x, n_bits=8):
        q, s = real(x, n_bits)
        q = q.copy()
        q.flat[0] = np.int8(np.clip(int(q.flat[0]) + 1, -127, 127)) if q.flat[0] < 127 else np.int8(126)
        return q, s
    codes._quant_rows = off_by_one
    with pytest.raises(AssertionError):
        encoder_chain(oracle_model, fx["src2"], fx["src_mask2"], codes)


def test_cfg2_teacher_forced_tokens(fx, oracle_model):
    """The oracle (not replayed) teacher-forced along the reference's cfg2 greedy path:
    its token differs from the reference's only where the reference's own margin over the
    oracle's pick is within the log-prob deviation the flips produce (2x its 99.9th
    percentile at agreeing positions), and the pick is among the reference's top 8."""
    om = oracle_model
    src, sm, ys = fx["src2"], fx["src_mask2"], fx["greedy2"]
    top8, top8_id = fx["top8"], fx["top8_id"]
    mem = om.encode(om.embed(src, om.src_lut), sm)
    st = O.DecodeState(om, mem, sm, ys.shape[1])
    B, T = ys.shape[0], ys.shape[1] - 1
    pred = np.zeros((B, T), np.int64)
    lp_at = np.zeros((B, T, 8), f32)
    for t in range(T):
        out = st.step(om.embed(ys[:, t:t + 1], om.tgt_lut, pos0=t))
        lp, nxt = om.generator(out)
        pred[:, t] = nxt
        lp_at[:, t] = np.take_along_axis(lp, top8_id[:, t], axis=1)
    ref = ys[:, 1:]
    np.testing.assert_array_equal(top8_id[..., 0], ref)
    dev = np.abs(lp_at - top8)
    agree = pred == ref
    bound = 2 * np.quantile(dev[agree], 0.999)
    print(f"cfg2 teacher-forced agreement {agree.mean():.4f} ({(~agree).sum()} of {agree.size}); "
          f"log-prob deviation p99.9 {bound / 2:.2e}")
    assert agree.mean() > 0.9
    for b, t in np.argwhere(~agree):
        k = np.nonzero(top8_id[b, t] == pred[b, t])[0]
        assert len(k), f"({b},{t}): oracle token outside the reference's top 8"
        assert top8[b, t, 0] - top8[b, t, k[0]] <= bound
