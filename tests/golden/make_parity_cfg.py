"""Generate tests/golden/golden_parity_cfg.npz: reference-replay fixtures at the BASELINE
shapes (tests/test_parity_cfg.py), from the REFERENCE's own modules.

Run in the build container only (it imports /root/reference, which never travels):

    python tests/golden/make_parity_cfg.py

Same model construction as make_golden.py.  Three workloads:

* cfg3 encoder: 4 sentences, lengths 100..128 padded to S = 128 (BASELINE cfg3's shape).
* cfg2: 8 sentences, lengths 24..64 padded to S = 72; the reference's batched greedy
  decode (71 steps, full-prefix recompute, first-index argmax) and its top-8 log-probs
  per step; then its decoder teacher-forced over the whole greedy prefix (T = 71).
* golden_model.npz's encoder and decoder module pass (so tests/test_oracle_golden.py's
  module tests replay instead of bounding the free-running deviation).

Per pass (cfg3 encoder, cfg2 encoder, cfg2 decoder, golden_model encoder / decoder) the
fixture holds the reference's rounding decisions in the sparse form of replay_codes.Codes
(the differences from the oracle's codes in the replayed state + a CRC-32 of every
reference code array) and every 16th row of the reference's per-layer outputs.  Written: data only, no reference source.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, REPO, os.path.join(REPO, "onnx-transformer_amd")]

from make_golden import REF, SEED, build_reference_model, import_reference  # noqa: E402
from make_parity import Recorder  # noqa: E402
from replay_codes import Codes, decoder_chain, encoder_chain, sample_rows  # noqa: E402


def sentences(rng, B, S, lo, hi):
    src = np.full((B, S), 2, np.int64)
    for b, n in enumerate(rng.integers(lo, hi + 1, B)):
        src[b, 0] = 0
        src[b, 1:n - 1] = rng.integers(4, 5337, n - 2)
        src[b, n - 1] = 1
    return src, (src != 2)[:, None, :]


def ref_encoder_layers(m, rec, src, sm, T):
    x = m.src_embed(T(src))
    outs = [x.numpy()]
    rec.on = True
    for layer in m.encoder.layers:
        x = layer(x, T(sm))
        outs.append(x.numpy())
    rec.on = False
    mem = m.encoder.norm(x)
    outs.append(mem.numpy())
    return outs, mem, rec.take(src.shape[0])


def ref_decoder_layers(m, rec, ys, mem, sm, T, tm):
    y = m.tgt_embed(T(ys))
    outs = [y.numpy()]
    rec.on = True
    for layer in m.decoder.layers:
        y = layer(y, mem, T(sm), tm)
        outs.append(y.numpy())
    rec.on = False
    outs.append(m.decoder.norm(y).numpy())
    return outs, rec.take(ys.shape[0])


def main():
    import torch
    torch.set_grad_enabled(False)
    from oracle.qtx_oracle import OracleModel
    from qtx.weights import synthetic_state_dict

    ref = import_reference()
    sd = synthetic_state_dict(SEED, ln_random=True)
    m = build_reference_model(ref, sd)
    om = OracleModel(sd)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    rng = np.random.default_rng(23)
    out = {}

    def oracle_pass(name, ref_codes, ref_outs, run):
        codes = Codes(ref=ref_codes)
        outs = run(codes)
        assert codes.i == len(ref_codes), f"{name}: {codes.i} oracle calls, {len(ref_codes)} reference"
        devs = [float(np.abs(sample_rows(a) - sample_rows(b)).max() / np.abs(sample_rows(b)).max())
                for a, b in zip(outs, ref_outs)]
        print(f"{name}: {len(ref_codes)} calls, {sum(codes.flips)} flips at {sum(codes.ties)} "
              f"near-ties; per-layer rel dev {['%.1e' % d for d in devs]}", flush=True)
        out.update(codes.pack(name))
        out[f"{name}_layers"] = np.stack([sample_rows(b) for b in ref_outs])
        return outs

    rec = Recorder(ref)
    rec.attach(m)

    # ---- cfg3 encoder: 4 x S = 128 -------------------------------------------------------
    src3, sm3 = sentences(rng, 4, 128, 100, 128)
    outs3, _, q3 = ref_encoder_layers(m, rec, src3, sm3, T)
    out.update(src3=src3, src_mask3=sm3)
    oracle_pass("enc3", q3, outs3, lambda c: encoder_chain(om, src3, sm3, c))

    # ---- cfg2: 8 x S = 72, greedy decode, teacher-forced decoder over T = 71 -------------
    src2, sm2 = sentences(rng, 8, 72, 24, 64)
    outs2, mem_ref, q2 = ref_encoder_layers(m, rec, src2, sm2, T)
    out.update(src2=src2, src_mask2=sm2)
    o_enc2 = oracle_pass("enc2", q2, outs2, lambda c: encoder_chain(om, src2, sm2, c))

    ys = torch.zeros((8, 1), dtype=torch.int64)
    top8, top8_id = [], []
    for _ in range(71):
        o = m.decode(mem_ref, T(sm2), ys, ref.utils.subsequent_mask(ys.size(1)).long())
        lp = m.generator(o[:, -1])
        v, i = torch.topk(lp, 8, dim=1)
        _, nxt = torch.max(lp, dim=1)
        assert (lp.gather(1, nxt[:, None])[:, 0] == v[:, 0]).all()
        top8.append(v.numpy())
        top8_id.append(i.numpy())
        ys = torch.cat([ys, nxt.unsqueeze(1)], dim=1)
    out.update(greedy2=ys.numpy(), top8=np.stack(top8, 1), top8_id=np.stack(top8_id, 1))

    dys = ys[:, :71].numpy()
    douts, qd = ref_decoder_layers(m, rec, dys, mem_ref, sm2, T, ref.utils.subsequent_mask(71).long())
    oracle_pass("dec2", qd, douts, lambda c: decoder_chain(om, dys, o_enc2[-1], sm2, c))

    # ---- golden_model.npz's module pass (2 x S = 16, decoder T = 8 on the reference
    # memory): replayed, tests/test_oracle_golden.py's module tests hold to fp32 noise ----
    gm = dict(np.load(os.path.join(HERE, "golden_model.npz")))
    gouts, gmem, qg = ref_encoder_layers(m, rec, gm["src"], gm["src_mask"], T)
    assert np.array_equal(gouts[-1], gm["memory"])
    oracle_pass("gm_enc", qg, gouts, lambda c: encoder_chain(om, gm["src"], gm["src_mask"], c))
    gdouts, qgd = ref_decoder_layers(m, rec, gm["ys"], gmem, gm["src_mask"], T, T(gm["tgt_mask"]))
    assert np.array_equal(gdouts[-1], gm["dec_out"])
    oracle_pass("gm_dec", qgd, gdouts, lambda c: decoder_chain(om, gm["ys"], gm["memory"], gm["src_mask"], c))

    np.savez_compressed(os.path.join(HERE, "golden_parity_cfg.npz"), **out)
    print({k: v.shape for k, v in out.items() if not k.endswith(("_idx", "_val"))}, "reference:", REF)


if __name__ == "__main__":
    main()
