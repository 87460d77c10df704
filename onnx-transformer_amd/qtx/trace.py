"""Op-by-op traced executor: the reference's node-by-node ONNX executor, which stores every
intermediate tensor in ``weight_dict`` by its graph name (onnx_optimized_inference.py:
32-57, 300-301), on the GPU through the per-op C-ABI entry points.

The fused product path (qtx_encoder_forward / qtx_decoder_forward) never materializes
the int8 codes of every quantizer or the MatMul accumulators.  ``trace_encoder`` /
``trace_decoder`` run the same arithmetic as separate launches (LayerNorm+quant, int8
GEMM, row quant, attention: the same kernels' parity-tested entry points, so the traced
output equals the fused output bit for bit) and hand back every quantizer's codes and
every QuantLinear MatMul's accumulators under the exported graphs' names:

* ``Round_<n>_out0``  the integer codes round(x / s) of a quantizer, float32 (as the
  graph's Round node outputs them), activations [B, S, K]; weights [K, N] (the MatMul's B
  operand) when ``weights=True``.  ``Round_<n>_scale``: the per-token / per-channel scale
  (a qtx addition: the graph keeps it in the following Mul).
* ``MatMul_<n>_out0``  float32(sum_k codes_x * codes_w) of a QuantLinear MatMul (exact
  integer below 2^24), [B, S, N].
* The attention MatMuls (campaign targets "FirstMatMul" / "SecondMatMul",
  input/encoder/matmul_3.json): ``MatMul_<QK>_out0`` = float32(sum_d q_codes * k_codes)
  per head [B, H, Sq, Sk] (the exact integer accumulators, before the / 8 and the mask, as
  for the QuantLinears); ``Round_<P>_out0`` = rint(P * 127) [B, H, Sq, Sk] (the Round of
  attention.py:33-35; ``Round_<P>_scale`` = 1/127); ``MatMul_<PV>_out0`` = the per-head
  context [B, H, Sq, 64] (fp32, the canonical PV chain).

Names follow the campaign target files input/{encoder,decoder}/matmul_*.json (e.g.
encoder MatMul_6 = Round_42_out0 x Round_4_out0), see :func:`encoder_names` /
:func:`decoder_names`.  The attention intermediates come from qtx_attention_trace (one wave
per query row and head, the canonical order): its context equals the fused attention's bit
for bit.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .model import _ptr, _stream

D = 512


# ---- graph names ----------------------------------------------------------------------

def encoder_names(L: int) -> dict:
    """Encoder layer L of encoder_try_cleaned.onnx: weight Rounds 6L+{Q,K,V,O,W1,W2},
    activation Rounds 36+8L+{in, q, k, v, P, ctx, ffn1_in, ffn2_in}, MatMul_{8L+i}."""
    a = 36 + 8 * L
    w = 6 * L
    return dict(
        act={"in": a, "q": a + 1, "k": a + 2, "v": a + 3, "P": a + 4, "ctx": a + 5,
             "ffn1_in": a + 6, "ffn2_in": a + 7},
        weight={"Q": w, "K": w + 1, "V": w + 2, "O": w + 3, "FFN1": w + 4, "FFN2": w + 5},
        matmul={"Q": 8 * L, "K": 8 * L + 1, "V": 8 * L + 2, "QK": 8 * L + 3, "PV": 8 * L + 4,
                "O": 8 * L + 5, "FFN1": 8 * L + 6, "FFN2": 8 * L + 7})


def decoder_names(L: int, n_layers: int = 6) -> dict:
    """Decoder layer L of decoder_try_cleaned.onnx: weight Rounds 10L+{Q,K,V,O,CQ,CK,CV,CO,
    W1,W2}; the memory quantizer Round_{10N} and the memory K/V outputs Round_{10N+1+2L},
    Round_{10N+2+2L}; layer activations Round_{10N+13+12L}+{in, q, k, v, P, ctx, c_in,
    c_q, c_P, c_ctx, ffn1_in, ffn2_in} (layer 0 numbers P before v); MatMul_{2L} /
    MatMul_{2L+1} memory K / V, MatMul_{2N+12L+i} the layer's own."""
    m0 = 10 * n_layers
    a = m0 + 13 + 12 * L
    act = {"in": a, "q": a + 1, "k": a + 2, "v": a + 3, "P": a + 4, "ctx": a + 5,
           "c_in": a + 6, "c_q": a + 7, "c_P": a + 8, "c_ctx": a + 9, "ffn1_in": a + 10,
           "ffn2_in": a + 11, "mem": m0, "c_k": m0 + 1 + 2 * L, "c_v": m0 + 2 + 2 * L}
    if L == 0:
        act["v"], act["P"] = a + 4, a + 3
    w = 10 * L
    b = 2 * n_layers + 12 * L
    return dict(
        act=act,
        weight={"Q": w, "K": w + 1, "V": w + 2, "O": w + 3, "CQ": w + 4, "CK": w + 5,
                "CV": w + 6, "CO": w + 7, "FFN1": w + 8, "FFN2": w + 9},
        matmul={"CK": 2 * L, "CV": 2 * L + 1, "Q": b, "K": b + 1, "V": b + 2, "QK": b + 3,
                "PV": b + 4, "O": b + 5, "CQ": b + 6, "CQK": b + 7, "CPV": b + 8, "CO": b + 9,
                "FFN1": b + 10, "FFN2": b + 11})


# ---- the executor ---------------------------------------------------------------------

class _Tracer:
    def __init__(self, model, rows_hint, weights):
        import torch
        self.torch, self.m, self.weights = torch, model, weights
        self.dev = model.device
        self.st = _stream(self.dev)
        self.wb = model.cfg.weight_bits
        self.out = {}
        n = 2048
        self.ones = torch.ones(max(rows_hint, n), device=self.dev)
        self.zeros = torch.zeros(n, device=self.dev)

    def linear(self, module, layer, idx):
        q, s, b = C.c_void_p(), C.c_void_p(), C.c_void_p()
        N, K = C.c_int32(), C.c_int32()
        _lib.call("qtx_model_linear", self.m.handle, module, layer, idx, C.byref(q), C.byref(s),
                  C.byref(b), C.byref(N), C.byref(K))
        return q, s, b, N.value, K.value

    def norm(self, module, layer, sub):
        a, b = C.c_void_p(), C.c_void_p()
        _lib.call("qtx_model_norm", self.m.handle, module, layer, sub, C.byref(a), C.byref(b))
        return a, b

    def empty(self, *shape, dtype=None):
        return self.torch.empty(shape, dtype=dtype or self.torch.float32, device=self.dev)

    def put_codes(self, n, q, s, shape):
        self.out[f"Round_{n}_out0"] = q.reshape(shape).float().cpu().numpy()
        self.out[f"Round_{n}_scale"] = s.reshape(shape[:-1] + (1,)).cpu().numpy()

    def quant(self, x, rows, K):
        q = self.empty(rows, K, dtype=self.torch.int8)
        s = self.empty(rows)
        _lib.call("qtx_row_quant", _ptr(x), rows, K, C.c_float(127.0), _ptr(q), _ptr(s), self.st)
        return q, s

    def ln_quant(self, x, rows, a, b):
        q = self.empty(rows, D, dtype=self.torch.int8)
        s = self.empty(rows)
        _lib.call("qtx_layernorm_quant", _ptr(x), a, b, rows, D, C.c_void_p(0), _ptr(q),
                  _ptr(s), self.st)
        return q, s

    def gemm(self, xq, xs, lin, rows, flags=0, res=None, mm=None, wname=None, shape=None):
        """One W8A8Linear: y = epilogue(xq . W^T); optionally its accumulators (unit
        scales, zero bias: exactly float(acc)) as MatMul_<mm>_out0."""
        W, sw, bias, N, K = lin
        y = self.empty(rows, N)
        _lib.call("qtx_linear_i8", _ptr(xq), _ptr(xs), W, sw, bias, rows, N, K, self.wb, flags,
                  _ptr(res), _ptr(y), self.st)
        if mm is not None:
            acc = self.empty(rows, N)
            _lib.call("qtx_linear_i8", _ptr(xq), _ptr(self.ones), W, _ptr(self.ones),
                      _ptr(self.zeros), rows, N, K, self.wb, 0, C.c_void_p(0), _ptr(acc), self.st)
            self.out[f"MatMul_{mm}_out0"] = acc.reshape(shape[:-1] + (N,)).cpu().numpy()
        if self.weights and wname is not None:
            self.put_weight(wname, W, sw, N, K)
        return y

    def put_weight(self, n, W, sw, N, K):
        """The model's quantized weight (codes [N, K], int4 unpacked) as the MatMul's B
        operand [K, N], and its per-channel scale."""
        torch = self.torch
        kb = K if self.wb == 8 else K // 2
        w = _view(torch, W.value, (N, kb), "|i1", self.dev).clone()
        if self.wb == 4:            # two's-complement nibbles, low nibble = even k
            w16 = w.to(torch.int16)
            w = torch.stack([(w16 << 12) >> 12, (w16 << 8) >> 12], -1).reshape(N, K)
        self.out[f"Round_{n}_out0"] = w.float().t().contiguous().cpu().numpy()
        self.out[f"Round_{n}_scale"] = _view(torch, sw.value, (N,), "<f4", self.dev).cpu().numpy()

    def attention(self, q, sq, k, sk, v, sv, mask, m_bs, m_is, B, Sq, Sk, names, dec=False):
        """Attention core with its intermediates stored under names = (Round of P,
        MatMul QK^T, MatMul PV); dec: a decoder layer's (the decoder's PV order)."""
        H = 8
        ctx = self.empty(B * Sq, D)
        qk = self.empty(B, H, Sq, Sk)
        pc = self.empty(B, H, Sq, Sk)
        _lib.call("qtx_attention_trace", _ptr(q), _ptr(sq), _ptr(k), _ptr(sk), _ptr(v),
                  _ptr(sv), _ptr(mask), m_bs, m_is, B, H, Sq, Sk, _ptr(ctx), _ptr(qk), _ptr(pc),
                  int(dec), self.st)
        p_n, qk_n, pv_n = names
        self.out[f"Round_{p_n}_out0"] = pc.cpu().numpy()
        self.out[f"Round_{p_n}_scale"] = np.float32(1.0) / np.float32(127.0)
        self.out[f"MatMul_{qk_n}_out0"] = qk.cpu().numpy()
        self.out[f"MatMul_{pv_n}_out0"] = (ctx.reshape(B, Sq, H, D // H).permute(0, 2, 1, 3)
                                           .contiguous().cpu().numpy())
        return ctx


class _DevView:
    """A model-owned device buffer seen by torch without a copy (the CUDA array interface,
    which torch's ROCm build consumes as HIP memory)."""

    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = {"shape": shape, "typestr": typestr,
                                         "data": (ptr, False), "version": 2}


def _view(torch, ptr, shape, typestr, device):
    return torch.as_tensor(_DevView(ptr, shape, typestr), device=device)


def trace_encoder(model, x, src_mask_u8, weights: bool = False):
    """Encoder forward (encoder.py:14-18) op by op.  x [B,S,512] f32 and src_mask_u8
    [B,S] uint8 device tensors -> (memory [B,S,512] device tensor, {name: ndarray})."""
    B, S, _ = x.shape
    M = B * S
    t = _Tracer(model, M, weights)
    x = x.reshape(M, D).contiguous()
    mask = src_mask_u8.contiguous()
    for L in range(model.cfg.n_layers):
        nm = encoder_names(L)
        act, wt, mm = nm["act"], nm["weight"], nm["matmul"]
        shp = (B, S, D)
        xq, xs = t.ln_quant(x, M, *t.norm(0, L, 0))
        t.put_codes(act["in"], xq, xs, shp)
        qkv = []
        for i, n in enumerate("QKV"):
            y = t.gemm(xq, xs, t.linear(0, L, i), M, mm=mm[n], wname=wt[n], shape=shp)
            q, s = t.quant(y, M, D)
            t.put_codes(act[n.lower()], q, s, shp)
            qkv += [q, s]
        ctx = t.attention(*qkv, mask, S, 0, B, S, S, (act["P"], mm["QK"], mm["PV"]))
        cq, cs = t.quant(ctx, M, D)
        t.put_codes(act["ctx"], cq, cs, shp)
        x = t.gemm(cq, cs, t.linear(0, L, 3), M, flags=2, res=x, mm=mm["O"], wname=wt["O"],
                   shape=shp)
        fq, fs = t.ln_quant(x, M, *t.norm(0, L, 1))
        t.put_codes(act["ffn1_in"], fq, fs, shp)
        h = t.gemm(fq, fs, t.linear(0, L, 4), M, flags=1, mm=mm["FFN1"], wname=wt["FFN1"],
                   shape=shp)
        F = h.shape[1]
        hq, hs = t.quant(h, M, F)
        t.put_codes(act["ffn2_in"], hq, hs, (B, S, F))
        x = t.gemm(hq, hs, t.linear(0, L, 5), M, flags=2, res=x, mm=mm["FFN2"],
                   wname=wt["FFN2"], shape=(B, S, F))
    out = t.empty(M, D)
    a, b = t.norm(0, -1, 0)
    _lib.call("qtx_layernorm_quant", _ptr(x), a, b, M, D, _ptr(out), C.c_void_p(0),
              C.c_void_p(0), t.st)
    return out.reshape(B, S, D), t.out


def trace_decoder(model, y, memory, src_mask_u8, tgt_mask_u8, weights: bool = False):
    """Decoder forward (decoder.py:13-16) op by op, full prefix.  y [B,T,512], memory
    [B,S,512] f32, src_mask_u8 [B,S], tgt_mask_u8 [T,T] (or [B,T,T]) -> (out, names)."""
    B, T, _ = y.shape
    S = memory.shape[1]
    M, Mm = B * T, B * S
    t = _Tracer(model, max(M, Mm), weights)
    x = y.reshape(M, D).contiguous()
    mem = memory.reshape(Mm, D).contiguous()
    sm = src_mask_u8.contiguous()
    tm = tgt_mask_u8.contiguous()
    tm_bs = 0 if tm.dim() == 2 else T * T
    shp, mshp = (B, T, D), (B, S, D)
    memq, mems = t.quant(mem, Mm, D)
    t.put_codes(decoder_names(0, model.cfg.n_layers)["act"]["mem"], memq, mems, mshp)
    for L in range(model.cfg.n_layers):
        nm = decoder_names(L, model.cfg.n_layers)
        act, wt, mm = nm["act"], nm["weight"], nm["matmul"]
        # self-attention
        xq, xs = t.ln_quant(x, M, *t.norm(1, L, 0))
        t.put_codes(act["in"], xq, xs, shp)
        qkv = []
        for i, n in enumerate("QKV"):
            yy = t.gemm(xq, xs, t.linear(1, L, i), M, mm=mm[n], wname=wt[n], shape=shp)
            q, s = t.quant(yy, M, D)
            t.put_codes(act[n.lower()], q, s, shp)
            qkv += [q, s]
        ctx = t.attention(*qkv, tm, tm_bs, T, B, T, T, (act["P"], mm["QK"], mm["PV"]), dec=True)
        cq, cs = t.quant(ctx, M, D)
        t.put_codes(act["ctx"], cq, cs, shp)
        x = t.gemm(cq, cs, t.linear(1, L, 3), M, flags=2, res=x, mm=mm["O"], wname=wt["O"],
                   shape=shp)
        # cross-attention on the memory
        xq, xs = t.ln_quant(x, M, *t.norm(1, L, 1))
        t.put_codes(act["c_in"], xq, xs, shp)
        yy = t.gemm(xq, xs, t.linear(1, L, 4), M, mm=mm["CQ"], wname=wt["CQ"], shape=shp)
        q, qs = t.quant(yy, M, D)
        t.put_codes(act["c_q"], q, qs, shp)
        kv = []
        for i, n in ((5, "CK"), (6, "CV")):
            yy = t.gemm(memq, mems, t.linear(1, L, i), Mm, mm=mm[n], wname=wt[n], shape=mshp)
            kq, ks = t.quant(yy, Mm, D)
            t.put_codes(act["c_k" if n == "CK" else "c_v"], kq, ks, mshp)
            kv += [kq, ks]
        ctx = t.attention(q, qs, *kv, sm, S, 0, B, T, S, (act["c_P"], mm["CQK"], mm["CPV"]), dec=True)
        cq, cs = t.quant(ctx, M, D)
        t.put_codes(act["c_ctx"], cq, cs, shp)
        x = t.gemm(cq, cs, t.linear(1, L, 7), M, flags=2, res=x, mm=mm["CO"], wname=wt["CO"],
                   shape=shp)
        # feed-forward
        fq, fs = t.ln_quant(x, M, *t.norm(1, L, 2))
        t.put_codes(act["ffn1_in"], fq, fs, shp)
        h = t.gemm(fq, fs, t.linear(1, L, 8), M, flags=1, mm=mm["FFN1"], wname=wt["FFN1"],
                   shape=shp)
        F = h.shape[1]
        hq, hs = t.quant(h, M, F)
        t.put_codes(act["ffn2_in"], hq, hs, (B, T, F))
        x = t.gemm(hq, hs, t.linear(1, L, 9), M, flags=2, res=x, mm=mm["FFN2"],
                   wname=wt["FFN2"], shape=(B, T, F))
    out = t.empty(M, D)
    a, b = t.norm(1, -1, 0)
    _lib.call("qtx_layernorm_quant", _ptr(x), a, b, M, D, _ptr(out), C.c_void_p(0),
              C.c_void_p(0), t.st)
    return out.reshape(B, T, D), t.out
