"""CPU ORACLE — test infrastructure only.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The product path
(``onnx-transformer_amd/qtx``) never imports it.

What it is: a numpy restatement of the reference's W8A8 inference arithmetic
(gebegebegebe/onnx-transformer).  The reference executes this arithmetic as fake-quant
fp32 graphs on ONNXRuntime-CPU; here it is restated as exact integer GEMMs
(int32 accumulators) plus a *canonical fp32 evaluation order* for every float step.
The canonical order is the contract the HIP kernels implement, so the GPU path and this
oracle agree bit-for-bit (see DESIGN.md §3 "numerics contract"):

* no FMA contraction except where the canonical order says ``fma`` (PV and generator dots;
  the generator's dot as four partial chains over k-quarters, summed pairwise; the
  decoder's PV as four partial chains over interleaved 4-key groups, attention_pv);
* LayerNorm / softmax / log-softmax sums use a fixed lane-split + xor-butterfly tree;
* softmax uses :func:`qexp`, a fixed polynomial exp that both sides evaluate identically.

Parity pinning: tests/test_oracle_golden.py checks this oracle against golden vectors
produced by importing the reference's own PyTorch modules (tests/golden/make_golden.py);
the ORT CPU path itself is unrunnable here, so ORT-level parity is unpinned.

The fma emulation (:func:`fma32`) is exact: float64 product and sum, with the
double-rounding case (the float64 sum exactly on a float32 midpoint) corrected from the
TwoSum error term.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32
EPS_SCALE = f32(1e-5)          # quant_linear.py:11,37 clamp(min=1e-5)
LN_EPS = f32(1e-6)             # layer_norm.py:6
MASK_FILL = f32(-1e9)          # attention.py:29
EXP_FLUSH = f32(-80.0)         # qexp() returns exactly 0 below this (keeps results normal)


# ---------------------------------------------------------------------------------------
# elementary canonical operations
# ---------------------------------------------------------------------------------------

def fma32(a, b, c):
    """Correctly rounded float32 fused multiply-add RN32(a*b + c), exact.

    a*b of two float32 is exact in float64; s = RN64(a*b + c) with the exact error e from
    TwoSum (a*b + c == s + e).  RN32(s) equals RN32(a*b + c) unless s is exactly a float32
    midpoint (the 29 mantissa bits below float32 precision read 1000...0) and e != 0
    (double rounding): then the result is the neighbour on e's side.  (Normal float32
    results; the callers' values are never subnormal.)"""
    p = np.asarray(a, np.float64) * np.asarray(b, np.float64)
    c = np.asarray(c, np.float64)
    s = p + c
    r = s.astype(f32)
    mid = (np.asarray(s).view(np.int64) & 0x1FFFFFFF) == 0x10000000
    if np.any(mid):
        bb = s - p
        e = (p - (s - bb)) + (c - bb)
        d = s - r.astype(np.float64)
        fix = mid & (e * d > 0)
        if np.any(fix):
            r = np.where(fix, np.nextafter(r, np.where(d > 0, f32(np.inf), f32(-np.inf))), r)
    return np.asarray(r, f32)


_H = lambda h: f32(float.fromhex(h))    # exact float32 constants, shared with qtx_common.h
_EXP_C = [_H("0x1.a01a02p-13"), _H("0x1.6c16c2p-10"), _H("0x1.111112p-7"),   # 1/7! .. 1/5!
          _H("0x1.555556p-5"), _H("0x1.555556p-3"), f32(0.5), f32(1.0), f32(1.0)]
_LOG2E = _H("0x1.715476p+0")
_LN2_HI = _H("0x1.62e4p-1")
_LN2_LO = _H("0x1.7f7d1cp-20")


def qexp(x):
    """Canonical fp32 exp: Cody-Waite reduction + degree-7 Taylor, Horner in fma.

    Mirrored exactly by ``qexp`` in onnx-transformer_amd/csrc/qtx_common.h.
    Inputs below -80 give exactly 0 (the softmax/log-softmax callers only need e^x for
    x <= 0, where such terms cannot change a 1/127-quantized probability).
    """
    x = np.asarray(x, f32)
    xc = np.maximum(x, f32(-100.0))
    n = np.rint(xc * _LOG2E).astype(f32)
    r = xc - n * _LN2_HI
    r = r - n * _LN2_LO
    p = np.full(r.shape, _EXP_C[0], f32)
    for c in _EXP_C[1:]:
        p = fma32(p, r, c)
    out = np.ldexp(p.astype(f32), n.astype(np.int32)).astype(f32)
    return np.where(x < EXP_FLUSH, f32(0.0), out).astype(f32)


def _butterfly(v):
    """Balanced pairwise tree over the 64 lane values in natural order — an xor-butterfly
    with offsets 1, 2, 4, ..., 32; returns lane 0.  The HIP side computes the same tree
    with DPP (qtx_common.h:wave_sum)."""
    v = np.asarray(v, f32)
    lanes = np.arange(v.shape[-1])
    off = 1
    while off < v.shape[-1]:
        v = v + v[..., lanes ^ off]
        off *= 2
    return v[..., 0]


def log_softmax_argmax(logits):
    """log_softmax over the last axis (generator.py:15) and torch.max's first index of the
    maximum (reference/onnx_reference_inference.py:640-641), in the canonical order:
    z = x - max, lse = log(lane-split sum of qexp(z)), logp = z - lse.
    Non-finite rows follow torch: a row holding a NaN or a +inf, or only -inf, has an
    all-NaN log_softmax (inf - inf, or a NaN that propagates), and torch.max of an all-NaN
    row is index 0 (pinned against torch in tests/test_oracle_golden.py).
    Returns (logp f32, ids int64)."""
    x = np.asarray(logits, f32)
    bad = np.isnan(x).any(-1) | np.isposinf(x).any(-1) | np.isneginf(x).all(-1)
    xs = np.where(bad[:, None], f32(0), x)
    m = xs.max(axis=-1)
    z = (xs - m[:, None]).astype(f32)
    lse = np.log(row_sum_lanesplit(qexp(z))).astype(f32)
    lp = (z - lse[:, None]).astype(f32)
    lp[bad] = np.nan
    ids = lp.argmax(axis=-1)
    ids[bad] = 0
    return lp, ids


def row_sum_lanesplit(x):
    """Sum over the last axis in the 'strided' canonical order.

    Lane l (0..63) accumulates x[l], x[l+64], x[l+128], ... starting from 0.0, then a
    64-lane xor-butterfly.  Used for softmax and log-softmax denominators.
    """
    x = np.asarray(x, f32)
    n = x.shape[-1]
    t = -(-n // 64)
    pad = np.zeros(x.shape[:-1] + (t * 64 - n,), f32)
    xp = np.concatenate([x, pad], axis=-1).reshape(x.shape[:-1] + (t, 64))
    acc = np.zeros(x.shape[:-1] + (64,), f32)
    for i in range(t):
        acc = acc + xp[..., i, :]
    return _butterfly(acc)


def row_sum_ln(x):
    """Sum over a row of D (multiple of 256) in the LayerNorm canonical order.

    Lane l owns the float4 chunks c = l, l+64, ... (elements 4c..4c+3); it sums its
    elements sequentially (chunk order, then element order), then xor-butterfly.
    """
    x = np.asarray(x, f32)
    D = x.shape[-1]
    nch = D // 256
    xc = x.reshape(x.shape[:-1] + (nch, 64, 4))
    acc = xc[..., 0, :, 0]
    for c in range(nch):
        for e in range(4):
            if c == 0 and e == 0:
                continue
            acc = acc + xc[..., c, :, e]
    return _butterfly(acc)


# ---------------------------------------------------------------------------------------
# quantizers — quant_linear.py
# ---------------------------------------------------------------------------------------

def quant_rows(x, n_bits: int = 8):
    """Per-row symmetric absmax quantizer.

    quant_linear.py:30-43 (per-token activations) and quant_linear.py:5-17 (per output
    channel weights) are the same formula on the last axis:
    ``s = clamp(max|x|, 1e-5) / q_max``, ``q = round_half_even(x / s)``; the reference
    returns ``q * s`` (fake quant), this returns the integers and the scale.
    """
    x = np.asarray(x, f32)
    qmax = f32(2 ** (n_bits - 1) - 1)
    s = np.maximum(np.abs(x).max(axis=-1), EPS_SCALE) / qmax
    q = np.rint(x / s[..., None])
    return q.astype(np.int8), s.astype(f32)


def dequant(q, s):
    """Fake-quant value ``q * s`` as the reference's quantizers return it."""
    return (np.asarray(q, f32) * np.asarray(s, f32)[..., None]).astype(f32)


def quant_weight(w, n_bits: int = 8):
    """quant_linear.py:5-17 — per output channel (rows of the nn.Linear weight)."""
    return quant_rows(w, n_bits)


# ---------------------------------------------------------------------------------------
# W8A8Linear — quant_linear.py:111-119
# ---------------------------------------------------------------------------------------

def int_gemm(qx, qw):
    """Exact int32 accumulators acc[m, n] = sum_k qx[m, k] * qw[n, k]."""
    a = np.asarray(qx, np.float64)
    b = np.asarray(qw, np.float64)
    acc = a @ b.T           # exact: |acc| <= K * 127^2 < 2^53
    return acc.astype(np.int64).astype(np.int32)


def linear_epilogue(acc, sx, sw, bias, relu=False):
    """y = ((float(acc) * s_x[m]) * s_w[n]) + b[n]   (+ ReLU, position_feed_forward.py:12)."""
    y = np.asarray(acc, np.int32).astype(f32)
    y = y * np.asarray(sx, f32)[..., :, None]
    y = y * np.asarray(sw, f32)
    y = y + np.asarray(bias, f32)
    if relu:
        y = np.where(y > 0, y, f32(0.0)).astype(f32)
    return y.astype(f32)


class QLinear:
    """Quantized weight of one W8A8Linear: int8 q [N, K], f32 s [N], f32 bias [N]."""

    def __init__(self, w, b, n_bits=8):
        self.q, self.s = quant_weight(w, n_bits)
        self.b = np.asarray(b, f32)

    def __call__(self, x, relu=False, quantize_output=False, fault=None):
        """W8A8Linear.forward (quant_linear.py:111-119) on an fp32 input x [..., K].

        fault (optional, fault-injection runs): dict with kind INPUT/INPUT16/WEIGHT/
        WEIGHT16/OUTPUT and row, col, bit, lo, hi, value in this linear's coordinates
        (rows = flattened tokens) — the reference's fault models
        (inject_utils/layers.py:48-84, onnx_optimized_inference.py:59-204): a bit-flipped
        int8 operand propagated through the MatMul (restricted to a window for *16), or
        one MatMul output (before bias) replaced by ``value``."""
        shp = x.shape
        qx, sx = quant_rows(x.reshape(-1, shp[-1]))
        acc = int_gemm(qx, self.q)
        if fault is not None and fault["kind"] != "OUTPUT":
            flip = lambda v: np.int8(np.uint8(np.int8(v).view(np.uint8) ^ (1 << fault["bit"])).view(np.int8))
            r, c, lo, hi = fault["row"], fault["col"], fault["lo"], fault["hi"]
            if fault["kind"].startswith("INPUT"):
                qx2 = qx.copy()
                qx2[r, c] = flip(qx2[r, c])
                acc2 = int_gemm(qx2, self.q)
                acc[r, lo:hi] = acc2[r, lo:hi]
            else:
                qw2 = self.q.copy()
                qw2[r, c] = flip(qw2[r, c])
                acc2 = int_gemm(qx, qw2)
                acc[lo:hi, r] = acc2[lo:hi, r]
        y = linear_epilogue(acc, sx, self.s, self.b)
        if fault is not None and fault["kind"] == "OUTPUT":
            y[fault["row"], fault["col"]] = f32(fault["value"]) + self.b[fault["col"]]
        if relu:
            y = np.where(y > 0, y, f32(0.0)).astype(f32)
        y = y.reshape(shp[:-1] + (y.shape[-1],))
        if quantize_output:          # get_quantized_model.py:160-168 (Q/K/V)
            return quant_rows(y)
        return y


# ---------------------------------------------------------------------------------------
# LayerNorm — layer_norm.py:12-15 (unbiased std, eps added to std)
# ---------------------------------------------------------------------------------------

def layer_norm(x, a, b):
    x = np.asarray(x, f32)
    D = x.shape[-1]
    mean = row_sum_ln(x) / f32(D)
    d = x - mean[..., None]
    var = row_sum_ln(d * d) / f32(D - 1)
    std = np.sqrt(var).astype(f32)
    den = std + LN_EPS
    y = (np.asarray(a, f32) * d) / den[..., None]
    return (y + np.asarray(b, f32)).astype(f32)


# ---------------------------------------------------------------------------------------
# attention — attention.py:23-36, on quantized Q/K/V (outputs of the QKV W8A8Linears)
# ---------------------------------------------------------------------------------------

def attention_scores(qq, sq, qk, sk, mask):
    """scores[b,h,i,j] = ((float(acc) * s_q[i]) * s_k[j]) / 8, masked_fill(mask==0, -1e9).

    qq [B,H,Sq,dk] int8, sq [B,Sq]; qk [B,H,Sk,dk], sk [B,Sk]; mask broadcastable to
    [B,Sq,Sk] (nonzero = keep).
    """
    acc = np.einsum("bhid,bhjd->bhij", qq.astype(np.int64), qk.astype(np.int64))
    s = acc.astype(np.int32).astype(f32)
    s = s * np.asarray(sq, f32)[:, None, :, None]
    s = s * np.asarray(sk, f32)[:, None, None, :]
    s = s / f32(8.0) if qq.shape[-1] == 64 else s / f32(np.sqrt(qq.shape[-1]))
    keep = np.broadcast_to(np.asarray(mask) != 0, (qq.shape[0], qq.shape[2], qk.shape[2]))
    return np.where(keep[:, None], s, MASK_FILL).astype(f32)


def softmax_quant(scores):
    """softmax(-1) then P = round(P*127)/127 (attention.py:30,33-35). Returns int P*127."""
    m = scores.max(axis=-1)
    e = qexp(scores - m[..., None])
    den = row_sum_lanesplit(e)
    p = e / den[..., None]
    return np.rint(p * f32(127.0)).astype(np.int8)


def attention_pv(qp, qv, sv, dec=False):
    """The PV MatMul (attention.py:36) in the canonical order.

    Encoder (dec=False): ctx[b,h,i,d] = one fma chain over j in key order, from 0, of
    (qp/127) * (float(qv) * s_v[j]).

    Decoder (dec=True, round 6; self and cross attention of decoder.py:28-33): four partial
    chains — chain c takes the keys j with (j >> 2) & 3 == c, in key order, from 0 — of the
    term fma(RN(P_j * s_v[j]), float(v_jd), acc_c), summed ((c0 + c1) + (c2 + c3)).  The
    decode step runs its PV as one lane per head dim (qtx_decode.hip k_dec_attn), where the
    single chain was a dependent fma per key; the chain split (keys 4 at a time, so one
    v_mfma_f32_16x16x4f32 step of the decoder-module kernel is one chain's 4 keys) and the
    per-key P * s_v product (one multiply per key instead of one per key and dim) shorten it.
    Same reference arithmetic (P @ (v * s_v) in fp32), a different rounding order."""
    P = qp.astype(f32) / f32(127.0)                                 # [B,H,Sq,Sk]
    B, H, Sq, Sk = P.shape
    if not dec:
        V = qv.astype(f32) * np.asarray(sv, f32)[:, None, :, None]  # [B,H,Sk,dk]
        acc = np.zeros((B, H, Sq, V.shape[-1]), f32)
        for j in range(Sk):
            acc = fma32(P[..., j, None], V[:, :, j, None, :], acc)
        return acc
    PS = (P * np.asarray(sv, f32)[:, None, None, :]).astype(f32)   # RN(P_j * s_v[j])
    V = qv.astype(f32)                                              # exact
    acc = [np.zeros((B, H, Sq, V.shape[-1]), f32) for _ in range(4)]
    for j in range(Sk):
        c = (j >> 2) & 3
        acc[c] = fma32(PS[..., j, None], V[:, :, j, None, :], acc[c])
    return ((acc[0] + acc[1]) + (acc[2] + acc[3])).astype(f32)


def split_heads(q, H):
    B, S, D = q.shape
    return q.reshape(B, S, H, D // H).transpose(0, 2, 1, 3)


def merge_heads(x):
    B, H, S, dk = x.shape
    return x.transpose(0, 2, 1, 3).reshape(B, S, H * dk)


def _flip8(v, bit):
    """flip_int8_bit (inject_utils/layers.py:62-69) on int8 storage."""
    return np.int8(np.uint8(np.int8(v).view(np.uint8) ^ (1 << int(bit))).view(np.int8))


def attention(qq, sq, qk, sk, qv, sv, mask, H=8, fault=None, dec=False):
    """Quantized Q/K/V [B,S,512] int8 + per-token scales -> ctx [B,Sq,512] f32, P ints.
    dec: the decoder's PV order (attention_pv).

    fault (fault-injection runs, one (sentence b, head h)): dict with kind QK_INPUT /
    QK_WEIGHT / QK_OUTPUT / PV_INPUT / PV_WEIGHT / PV_OUTPUT and b, h, i, j, d, lo, hi,
    bit, value (the conventions of include/qtx.h): a flipped q / k element changes the
    exact int QK^T accumulators (INPUT: keys lo..hi of row i, WEIGHT: rows lo..hi of key
    j); a flipped P*127 int / v element is used by the PV chain (INPUT: dims lo..hi of row
    i, WEIGHT: rows lo..hi of dim d); OUTPUT replaces the QK^T value (before / 8 and the
    mask) or the context value."""
    q4, k4, v4 = split_heads(qq, H), split_heads(qk, H), split_heads(qv, H)
    if fault is None:
        scores = attention_scores(q4, sq, k4, sk, mask)
        qp = softmax_quant(scores)
        ctx = attention_pv(qp, v4, sv, dec)
        return merge_heads(ctx), qp
    kind, b, h = fault["kind"], fault["b"], fault["h"]
    i, j, d, lo, hi, bit = (fault[k] for k in ("i", "j", "d", "lo", "hi", "bit"))
    acc = np.einsum("bhid,bhjd->bhij", q4.astype(np.int64), k4.astype(np.int64))
    if kind == "QK_INPUT":
        dq = int(_flip8(q4[b, h, i, d], bit)) - int(q4[b, h, i, d])
        acc[b, h, i, lo:hi] += dq * k4[b, h, lo:hi, d].astype(np.int64)
    elif kind == "QK_WEIGHT":
        dk = int(_flip8(k4[b, h, j, d], bit)) - int(k4[b, h, j, d])
        acc[b, h, lo:hi, j] += q4[b, h, lo:hi, d].astype(np.int64) * dk
    s = acc.astype(np.int32).astype(f32)
    s = s * np.asarray(sq, f32)[:, None, :, None]
    s = s * np.asarray(sk, f32)[:, None, None, :]
    s = s / f32(8.0)
    if kind == "QK_OUTPUT":
        s[b, h, i, j] = f32(fault["value"]) / f32(8.0)
    keep = np.broadcast_to(np.asarray(mask) != 0, (q4.shape[0], q4.shape[2], k4.shape[2]))
    scores = np.where(keep[:, None], s, MASK_FILL).astype(f32)
    qp = softmax_quant(scores)
    ctx = attention_pv(qp, v4, sv, dec)
    if kind == "PV_INPUT":
        qp2 = qp[b:b + 1, h:h + 1].copy()
        qp2[0, 0, i, j] = _flip8(qp2[0, 0, i, j], bit)
        c2 = attention_pv(qp2, v4[b:b + 1, h:h + 1], np.asarray(sv)[b:b + 1], dec)
        ctx[b, h, i, lo:hi] = c2[0, 0, i, lo:hi]
    elif kind == "PV_WEIGHT":
        v2 = v4[b:b + 1, h:h + 1].copy()
        v2[0, 0, j, d] = _flip8(v2[0, 0, j, d], bit)
        c2 = attention_pv(qp[b:b + 1, h:h + 1], v2, np.asarray(sv)[b:b + 1], dec)
        ctx[b, h, lo:hi, d] = c2[0, 0, lo:hi, d]
    elif kind == "PV_OUTPUT":
        ctx[b, h, i, d] = f32(fault["value"])
    return merge_heads(ctx), qp


# ---------------------------------------------------------------------------------------
# model
# ---------------------------------------------------------------------------------------

class OracleModel:
    """Quantized model restated from the reference modules (model.py:15-37)."""

    def __init__(self, sd, n_layers=6, n_heads=8, n_bits=8):
        self.N, self.H = n_layers, n_heads
        L = lambda p: QLinear(sd[p + ".weight"], sd[p + ".bias"], n_bits)
        Nm = lambda p: (np.asarray(sd[p + ".a_2"], f32), np.asarray(sd[p + ".b_2"], f32))
        self.enc = []
        for i in range(n_layers):
            p = f"encoder.layers.{i}"
            self.enc.append(dict(
                attn=[L(f"{p}.self_attn.linears.{j}") for j in range(4)],
                w1=L(f"{p}.feed_forward.w_1"), w2=L(f"{p}.feed_forward.w_2"),
                ln=[Nm(f"{p}.sublayer.{j}.norm") for j in range(2)]))
        self.enc_norm = Nm("encoder.norm")
        self.dec = []
        for i in range(n_layers):
            p = f"decoder.layers.{i}"
            self.dec.append(dict(
                self_attn=[L(f"{p}.self_attn.linears.{j}") for j in range(4)],
                src_attn=[L(f"{p}.src_attn.linears.{j}") for j in range(4)],
                w1=L(f"{p}.feed_forward.w_1"), w2=L(f"{p}.feed_forward.w_2"),
                ln=[Nm(f"{p}.sublayer.{j}.norm") for j in range(3)]))
        self.dec_norm = Nm("decoder.norm")
        self.src_lut = np.asarray(sd["src_embed.0.lut.weight"], f32)
        self.tgt_lut = np.asarray(sd["tgt_embed.0.lut.weight"], f32)
        self.pe = np.asarray(sd["src_embed.1.pe"], f32).reshape(-1, self.src_lut.shape[1])
        self.gen_w = np.asarray(sd["generator.proj.weight"], f32)
        self.gen_b = np.asarray(sd["generator.proj.bias"], f32)

    # -- fault injection ---------------------------------------------------------------
    @staticmethod
    def _lin_fault(fault, module, layer, linear, rows, n_out):
        """The fault (qtx.fault.Fault-like dict) as a QLinear fault dict if it targets this
        linear, else None.  Windows: INPUT16 columns, WEIGHT16 rows."""
        if (fault is None or fault["module"] != module or fault["layer"] != layer
                or fault["linear"] != linear):
            return None
        k = fault["kind"]
        kind = "OUTPUT" if k.startswith("RANDOM") or k == "OUTPUT" else k
        if kind in ("INPUT16", "WEIGHT16"):
            lo, hi = fault["win_start"], fault["win_start"] + fault["win_len"]
        else:
            lo, hi = 0, (n_out if kind == "INPUT" else rows)
        return dict(kind=kind, row=fault["row"], col=fault["col"], bit=fault.get("bit", 0),
                    lo=lo, hi=hi, value=fault.get("value", 0.0))

    # -- sublayers ---------------------------------------------------------------------
    @staticmethod
    def _attn_fault(fault, module, layer, qk_name, pv_name, Sq, Sk):
        """The fault as an oracle attention() fault dict if it targets this attention's
        QK^T (qk_name) or PV (pv_name) MatMul, else None (index conventions: qtx.h)."""
        if (fault is None or fault["module"] != module or fault["layer"] != layer
                or fault["linear"] not in (qk_name, pv_name)):
            return None
        qk = fault["linear"] == qk_name
        k = fault["kind"]
        out = k.startswith("RANDOM") or k == "OUTPUT"
        inp = k.startswith("INPUT")
        win = k.endswith("16")
        r, c = fault["row"], fault["col"]
        f = dict(bit=fault.get("bit", 0), value=fault.get("value", 0.0), i=0, j=0, d=0, lo=0, hi=0)
        if out or inp:
            f["b"], f["i"] = divmod(r, Sq)
            if qk and inp:
                f["h"], f["d"] = divmod(c, 64)
            elif qk or inp:
                f["h"], f["j"] = divmod(c, Sk)
            else:
                f["h"], f["d"] = divmod(c, 64)
        else:
            f["b"], f["j"] = divmod(r, Sk)
            f["h"], f["d"] = divmod(c, 64)
        if out:
            f["kind"] = "QK_OUTPUT" if qk else "PV_OUTPUT"
        elif inp:
            f["kind"] = "QK_INPUT" if qk else "PV_INPUT"
            f["lo"], f["hi"] = ((fault["win_start"], fault["win_start"] + fault["win_len"]) if win
                                else (0, Sk if qk else 64))
        else:
            f["kind"] = "QK_WEIGHT" if qk else "PV_WEIGHT"
            f["lo"], f["hi"] = ((fault["win_start"], fault["win_start"] + fault["win_len"]) if win
                                else (0, Sq))
        return f

    def mha(self, lin, xq, xkv, mask, faults=(None,) * 4, attn_fault=None, dec=False):
        """MultiHeadedAttention.forward (attention.py:39-67); dec: a decoder layer's
        attention (the decoder's PV order, attention_pv)."""
        qq, sq = lin[0](xq, quantize_output=True, fault=faults[0])
        qk, sk = lin[1](xkv, quantize_output=True, fault=faults[1])
        qv, sv = lin[2](xkv, quantize_output=True, fault=faults[2])
        ctx, _ = attention(qq, sq, qk, sk, qv, sv, mask, self.H, fault=attn_fault, dec=dec)
        return lin[3](ctx, fault=faults[3])

    def ffn(self, lp, x, faults=(None, None)):
        """PositionwiseFeedForward.forward (position_feed_forward.py:11-12)."""
        return lp["w2"](lp["w1"](x, relu=True, fault=faults[0]), fault=faults[1])

    # -- stacks ------------------------------------------------------------------------
    def encode(self, x, src_mask, fault=None):
        """Encoder.forward (encoder.py:14-18, 29-32). x [B,S,512], src_mask [B,1,S].
        fault: optional dict (qtx.fault.Fault.as_dict()) with module 0."""
        x = np.asarray(x, f32)
        m = np.asarray(src_mask).reshape(x.shape[0], 1, -1)
        rows = x.shape[0] * x.shape[1]
        for L, lp in enumerate(self.enc):
            lf = lambda lin, n=512: self._lin_fault(fault, 0, L, lin, rows, n)
            h = layer_norm(x, *lp["ln"][0])
            S = x.shape[1]
            x = x + self.mha(lp["attn"], h, h, m, [lf("Q"), lf("K"), lf("V"), lf("O")],
                             self._attn_fault(fault, 0, L, "QK", "PV", S, S))
            x = x + self.ffn(lp, layer_norm(x, *lp["ln"][1]),
                             [lf("FFN1", lp["w1"].q.shape[0]), lf("FFN2")])
        return layer_norm(x, *self.enc_norm)

    def decode(self, y, memory, src_mask, tgt_mask, fault=None):
        """Decoder.forward (decoder.py:13-16, 28-33). tgt_mask [1|B,T,T].
        fault: optional dict (qtx.fault.Fault.as_dict()) with module 1."""
        x = np.asarray(y, f32)
        B = x.shape[0]
        sm = np.asarray(src_mask).reshape(B, 1, -1)
        tm = np.broadcast_to(np.asarray(tgt_mask), (B,) + np.asarray(tgt_mask).shape[-2:])
        rows, mrows = B * x.shape[1], B * np.asarray(memory).shape[1]
        for L, lp in enumerate(self.dec):
            lf = lambda lin, r=rows, n=512: self._lin_fault(fault, 1, L, lin, r, n)
            h = layer_norm(x, *lp["ln"][0])
            T, S = x.shape[1], np.asarray(memory).shape[1]
            x = x + self.mha(lp["self_attn"], h, h, tm, [lf("Q"), lf("K"), lf("V"), lf("O")],
                             self._attn_fault(fault, 1, L, "QK", "PV", T, T), dec=True)
            h = layer_norm(x, *lp["ln"][1])
            x = x + self.mha(lp["src_attn"], h, memory, sm,
                             [lf("CQ"), lf("CK", mrows), lf("CV", mrows), lf("CO")],
                             self._attn_fault(fault, 1, L, "CQK", "CPV", T, S), dec=True)
            x = x + self.ffn(lp, layer_norm(x, *lp["ln"][2]),
                             [lf("FFN1", rows, lp["w1"].q.shape[0]), lf("FFN2")])
        return layer_norm(x, *self.dec_norm)

    # -- host-side pieces of the decode loop ---------------------------------------------
    def embed(self, ids, lut, pos0=0):
        """Embeddings + PositionalEncoding (embeddings.py:12-13, positional_encodings.py:23-26)."""
        ids = np.asarray(ids)
        e = lut[ids] * f32(np.sqrt(512.0) if lut.shape[1] == 512 else np.sqrt(lut.shape[1]))
        return (e + self.pe[pos0:pos0 + ids.shape[1]][None]).astype(f32)

    def logits(self, x):
        """proj(x) of generator.py:15 in the canonical order: four partial fma chains, chain q
        sequential over k in [128q, 128q + 128) from 0, summed as ((c0 + c1) + (c2 + c3)),
        then + bias (round 5: the four chains run on four waves, qtx_decode.hip
        k_generator_mfma; the reference's fp32 Linear sums in MLAS order, pinned within 1e-5
        by tests/test_oracle_golden.py)."""
        x = np.asarray(x, f32)
        K = x.shape[1]
        kq = K // 4
        acc = [np.zeros((x.shape[0], self.gen_w.shape[0]), f32) for _ in range(4)]
        for q in range(4):
            for k in range(q * kq, (q + 1) * kq):
                acc[q] = fma32(x[:, k, None], self.gen_w[None, :, k], acc[q])
        return (((acc[0] + acc[1]) + (acc[2] + acc[3])) + self.gen_b).astype(f32)

    def generator(self, x):
        """Generator.forward (generator.py:14-15) + first-index argmax
        (reference/onnx_reference_inference.py:640-641).  Returns (logprobs, ids)."""
        return log_softmax_argmax(self.logits(x))

    def greedy_decode(self, src, src_mask, max_len=72, start=0, kv_cache=True, fault=None,
                      fault_step=0):
        """Batched greedy decode (batch_output.py:659-673; B=1 form
        reference/onnx_reference_inference.py:622-646): fixed max_len-1 steps, no EOS exit.

        kv_cache=False recomputes the whole prefix each step exactly like the reference;
        kv_cache=True computes only the new position (identical by causal invariance).
        """
        src = np.asarray(src)
        B = src.shape[0]
        enc_fault = fault if fault is not None and fault["module"] == 0 else None
        dec_fault = fault if fault is not None and fault["module"] == 1 else None
        memory = self.encode(self.embed(src, self.src_lut), src_mask, fault=enc_fault)
        ys = np.full((B, 1), start, np.int64)
        if not kv_cache or dec_fault is not None:
            # a decoder fault corrupts the decoder run of step fault_step only
            # (parallelized_inject_onnx_transformer.py:639: target_inference_number - 1)
            for i in range(max_len - 1):
                T = ys.shape[1]
                out = self.decode(self.embed(ys, self.tgt_lut), memory, src_mask,
                                  np.tril(np.ones((1, T, T), np.int64)),
                                  fault=dec_fault if i == fault_step else None)
                _, nxt = self.generator(out[:, -1])
                ys = np.concatenate([ys, nxt[:, None]], axis=1)
            return ys
        st = DecodeState(self, memory, src_mask, max_len)
        for t in range(max_len - 1):
            out = st.step(self.embed(ys[:, -1:], self.tgt_lut, pos0=t))
            _, nxt = self.generator(out)
            ys = np.concatenate([ys, nxt[:, None]], axis=1)
        return ys


class DecodeState:
    """KV-cached decoder: self-attn K/V appended per step, cross K/V computed once."""

    def __init__(self, model: OracleModel, memory, src_mask, max_len):
        self.m = model
        self.sm = np.asarray(src_mask).reshape(memory.shape[0], 1, -1)
        self.cross = [(lp["src_attn"][1](memory, quantize_output=True),
                       lp["src_attn"][2](memory, quantize_output=True)) for lp in model.dec]
        self.kcache = [None] * model.N
        self.vcache = [None] * model.N

    def step(self, y):
        """One new position per sentence: y [B,1,512] -> decoder output [B,512]."""
        m = self.m
        x = np.asarray(y, f32)
        B = x.shape[0]
        for L, lp in enumerate(m.dec):
            h = layer_norm(x, *lp["ln"][0])
            lin = lp["self_attn"]
            qq, sq = lin[0](h, quantize_output=True)
            k, v = lin[1](h, quantize_output=True), lin[2](h, quantize_output=True)
            if self.kcache[L] is None:
                self.kcache[L], self.vcache[L] = k, v
            else:
                self.kcache[L] = tuple(np.concatenate([a, b], 1) for a, b in zip(self.kcache[L], k))
                self.vcache[L] = tuple(np.concatenate([a, b], 1) for a, b in zip(self.vcache[L], v))
            (qk, sk), (qv, sv) = self.kcache[L], self.vcache[L]
            ones = np.ones((B, 1, qk.shape[1]), np.int64)
            ctx, _ = attention(qq, sq, qk, sk, qv, sv, ones, m.H, dec=True)
            x = x + lin[3](ctx)
            h = layer_norm(x, *lp["ln"][1])
            lin = lp["src_attn"]
            qq, sq = lin[0](h, quantize_output=True)
            (qk, sk), (qv, sv) = self.cross[L]
            ctx, _ = attention(qq, sq, qk, sk, qv, sv, self.sm, m.H, dec=True)
            x = x + lin[3](ctx)
            x = x + m.ffn(lp, layer_norm(x, *lp["ln"][2]))
        return layer_norm(x, *m.dec_norm)[:, 0]


def subsequent_mask(T):
    """utils.py:10-14 / reference/onnx_reference_inference.py:649-655 as int64 [1,T,T]."""
    return np.tril(np.ones((1, T, T), np.int64))
