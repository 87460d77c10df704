"""Generate the golden vectors in tests/golden/*.npz from the REFERENCE's own modules.

Run in the build container only (it needs /root/reference, which never travels):

    python tests/golden/make_golden.py

It imports the reference's PyTorch modules (quant_linear, attention, layer_norm,
encoder/decoder, model, get_quantized_model, ...) exactly as SURVEY §8c describes:
``brevitas``/``qonnx`` are stubbed in ``sys.modules`` (imported but unused on this path:
model.py:13, encoder_decoder.py:3-4, embeddings.py:3, generator.py:2-3), the model is
built with ``make_model``, passed through ``get_quantized`` and then ``load_state_dict``
(the order of output.py:609-613), with deterministic synthetic weights from
``qtx.weights.synthetic_state_dict``.  Only inputs and reference outputs are written
(data, no reference source).  The outputs are the reference's fake-quant fp32 values.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("QTX_REFERENCE", "/root/reference")
SEED = 20241223


def import_reference():
    for name in ["brevitas", "brevitas.nn", "brevitas.export", "brevitas.quant",
                 "brevitas.quant.scaled_int", "qonnx", "qonnx.core", "qonnx.core.modelwrapper"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["brevitas.export"].export_onnx_qcdq = None
    sys.modules["brevitas.quant.scaled_int"].Int32Bias = None
    sys.modules["qonnx.core.modelwrapper"].ModelWrapper = None
    sys.path.insert(0, REF)
    import attention
    attention.print = lambda *a, **k: None      # attention.py:40-48 prints every call
    import get_quantized_model
    import layer_norm
    import model
    import quant_linear
    import utils
    return types.SimpleNamespace(model=model, gq=get_quantized_model, ql=quant_linear,
                                 attention=attention, layer_norm=layer_norm, utils=utils)


def build_reference_model(ref, sd_np):
    import torch
    cwd = os.getcwd()
    os.chdir(REF)                       # get_quantized loads scales/transformer_scales.pt
    try:
        m = ref.model.make_model(5337, 4444, N=6)
        m = ref.gq.get_quantized(m)     # smoothing + W8A8Linear swap (get_quantized_model.py:174-178)
    finally:
        os.chdir(cwd)
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd_np.items()})
    m.eval()
    return m


def main():
    import torch
    torch.set_grad_enabled(False)
    sys.path.insert(0, os.path.join(REPO, "onnx-transformer_amd"))
    from qtx.weights import synthetic_state_dict

    ref = import_reference()
    sd = synthetic_state_dict(SEED, ln_random=True)
    m = build_reference_model(ref, sd)
    rng = np.random.default_rng(7)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    out = {}

    # ---- per-token quantizer (quant_linear.py:30-43) incl. edge rows --------------------
    xq = rng.standard_normal((8, 512)).astype(np.float32) * 3
    xq[0] = 0.0                                            # all-zero row -> clamp(1e-5)
    xq[1] = 0.0
    xq[1, :8] = [127.0, 0.5, 1.5, 2.5, -0.5, -1.5, -2.5, 126.5]  # exact half-way ties, s = 1
    xq[2] *= 1e-7                                          # tiny row, still above clamp
    xq[3] *= 1e-9                                          # below clamp
    out["quant_x"] = xq
    out["quant_ref"] = ref.ql.quantize_activation_per_token_absmax(T(xq), n_bits=8).numpy()
    w = sd["encoder.layers.0.feed_forward.w_1.weight"][:64]
    out["wquant_ref8"] = ref.ql.quantize_weight_per_channel_absmax(T(w), n_bits=8).numpy()
    out["wquant_ref4"] = ref.ql.quantize_weight_per_channel_absmax(T(w), n_bits=4).numpy()

    # ---- W8A8Linear forward per linear kind (quant_linear.py:111-119) -------------------
    lay = m.encoder.layers[0]
    x512 = rng.standard_normal((2, 24, 512)).astype(np.float32)
    out["lin_x512"] = x512
    out["lin_q_ref"] = lay.self_attn.linears[0](T(x512)).numpy()      # output-quantized (QKV)
    out["lin_o_ref"] = lay.self_attn.linears[3](T(x512)).numpy()      # O-proj
    out["lin_ffn_ref"] = lay.feed_forward(T(x512)).numpy()            # w_2(relu(w_1 x))
    h = torch.relu(lay.feed_forward.w_1(T(x512)))
    out["lin_ffn1_ref"] = h.numpy()
    out["lin_ffn2_ref"] = lay.feed_forward.w_2(h).numpy()

    # ---- LayerNorm (layer_norm.py:12-15) ------------------------------------------------
    xl = (rng.standard_normal((16, 512)) * rng.uniform(0.1, 10, (16, 1))).astype(np.float32)
    out["ln_x"] = xl
    out["ln_ref"] = lay.sublayer[0].norm(T(xl)).numpy()

    # ---- attention core (attention.py:23-36) on fake-quant Q/K/V ------------------------
    B, H, S, dk = 2, 8, 20, 64
    qi = rng.integers(-127, 128, (3, B, S, H * dk)).astype(np.int8)
    sc = rng.uniform(0.005, 0.05, (3, B, S)).astype(np.float32)
    deq = (qi.astype(np.float32) * sc[..., None]).astype(np.float32)
    split = lambda a: T(a.reshape(B, S, H, dk).transpose(0, 2, 1, 3).copy())
    mask = np.ones((B, 1, S), bool)
    mask[1, 0, 15:] = False
    ctx, p = lay.self_attn.attention(split(deq[0]), split(deq[1]), split(deq[2]),
                                     mask=T(mask).unsqueeze(1))
    out.update(attn_qi=qi, attn_sc=sc, attn_mask=mask, attn_ctx_ref=ctx.numpy(),
               attn_p_ref=p.numpy())

    # ---- embeddings + PE, generator ------------------------------------------------------
    ids = rng.integers(0, 5337, (2, 12))
    out["emb_ids"] = ids
    out["emb_ref"] = m.src_embed(T(ids)).numpy()
    out["pe_ref"] = m.src_embed[1].pe[0, :128].numpy()
    xg = rng.standard_normal((4, 512)).astype(np.float32)
    out["gen_x"] = xg
    out["gen_ref"] = m.generator(T(xg)).numpy()
    np.savez_compressed(os.path.join(HERE, "golden_ops.npz"), **out)

    # ---- module level: encoder, decoder, greedy decode ----------------------------------
    Bm, Sm = 2, 16
    src = np.full((Bm, Sm), 2, np.int64)                  # <blank> = 2 padding
    lens = [16, 11]
    for b, n in enumerate(lens):
        src[b, 0] = 0
        src[b, 1:n - 1] = rng.integers(4, 5337, n - 2)
        src[b, n - 1] = 1
    src_mask = (src != 2)[:, None, :]                      # batch.py:7
    memory = m.encode(T(src), T(src_mask))
    mod = dict(src=src, src_mask=src_mask, enc_in=m.src_embed(T(src)).numpy(),
               memory=memory.numpy())
    Tt = 8
    ys = rng.integers(4, 4444, (Bm, Tt))
    ys[:, 0] = 0
    tmask = ref.utils.subsequent_mask(Tt).long()
    dec = m.decode(memory, T(src_mask), T(ys), tmask)
    mod.update(ys=ys, dec_in=m.tgt_embed(T(ys)).numpy(), tgt_mask=tmask.numpy(),
               dec_out=dec.numpy())
    # batched greedy decode, batch_output.py:659-673 semantics (full prefix recompute)
    max_len = 72
    ysg = torch.full((Bm, 1), 0, dtype=torch.int64)
    for _ in range(max_len - 1):
        o = m.decode(memory, T(src_mask), ysg, ref.utils.subsequent_mask(ysg.size(1)).long())
        prob = m.generator(o[:, -1])
        _, nxt = torch.max(prob, dim=1)
        ysg = torch.cat([ysg, nxt.unsqueeze(1)], dim=1)
    mod["greedy"] = ysg.numpy()
    np.savez_compressed(os.path.join(HERE, "golden_model.npz"), **mod)
    print("wrote", sorted(out), sorted(mod))


if __name__ == "__main__":
    main()
