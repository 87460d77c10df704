"""The fused FFN sublayer (qtx_ffn_rows, csrc/qtx_ffn.hip k_ffn_fused) through the C-ABI,
bit-exact against the oracle: FFN1 + ReLU + per-token quantization of the hidden
(quant_linear.py:30-43 over all d_ff columns), FFN2 + residual (position_feed_forward.py:11-12,
sublayer_connection.py:15-17), then the next LayerNorm quantized (KP) or the final
LayerNorm in fp32 (layer_norm.py:12-15).  The stream packer (qtx_pack_ffn) is checked against
its layout restated in numpy."""
import ctypes as C

import numpy as np
import pytest

from oracle import qtx_oracle as O

pytestmark = pytest.mark.gpu
f32 = np.float32
P = C.c_void_p
S0 = C.c_void_p(0)
_KEEP = []


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def dev(torch, a):
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    _KEEP.append(t)
    return t


def to_kp(a):
    M, K = a.shape
    if M & 1:
        a = np.concatenate([a, np.zeros((1, K), a.dtype)])
    return np.ascontiguousarray(a.reshape(-1, 2, K // 64, 64).transpose(0, 2, 1, 3)).reshape(-1, K)


def from_kp(a, M):
    K = a.shape[1]
    return a.reshape(-1, K // 64, 2, 64).transpose(0, 2, 1, 3).reshape(-1, K)[:M]


def pack_ref(w1, w2):
    """qtx_pack_ffn's stream (include/qtx.h) restated: [F/64 chunks][4 slots][16 fragments]
    [64 lanes][16 bytes]; slots 0, 1 = W1 K steps 0-3 / 4-7, slots 2, 3 = W2 column half 0 / 1."""
    F = w1.shape[0]
    nc = F // 64
    out = np.zeros((nc, 4, 16, 64, 16), np.int8)
    lane = np.arange(64)
    f, g = lane & 15, lane >> 4
    b = np.arange(16)
    for c in range(nc):
        for fr in range(16):
            for hh in range(2):
                s, j = 4 * hh + (fr >> 2), fr & 3
                rows = w1[64 * c + 16 * j + f]                          # [64, 512]
                idx = 64 * s + 16 * g[:, None] + b[None, :]
                out[c, hh, fr] = np.take_along_axis(rows, idx, axis=1)
            for ch in range(2):
                col = np.where(fr < 8, 16 * f + 8 * ch + fr, 256 + 16 * f + 8 * ch + fr - 8)
                k = 64 * c + 16 * (b[None, :] >> 2) + 4 * g[:, None] + (b[None, :] & 3)
                out[c, 2 + ch, fr] = np.take_along_axis(w2[col], k, axis=1)
    return out.reshape(-1)


def test_pack_ffn(torch):
    from qtx._lib import lib
    rng = np.random.default_rng(3)
    for F in (2048, 256):
        w1 = rng.integers(-127, 128, (F, 512)).astype(np.int8)
        w2 = rng.integers(-127, 128, (512, F)).astype(np.int8)
        out = torch.empty(F * 1024, dtype=torch.int8, device="cuda")
        assert lib().qtx_pack_ffn(P(dev(torch, w1).data_ptr()), P(dev(torch, w2).data_ptr()), F,
                                  P(out.data_ptr()), S0) == 0
        np.testing.assert_array_equal(out.cpu().numpy(), pack_ref(w1, w2))
    assert lib().qtx_pack_ffn(P(dev(torch, w1).data_ptr()), P(dev(torch, w2).data_ptr()), 100,
                              P(out.data_ptr()), S0) == 4


def ffn_case(torch, M, F, lnq=True, scale_spread=False, seed=0, alias=False):
    from qtx._lib import FfnRows, lib
    rng = np.random.default_rng(seed + M + F)
    x1 = (rng.standard_normal((M, 512)) * 2).astype(f32)
    la = (1 + 0.1 * rng.standard_normal(512)).astype(f32)
    lb = (0.1 * rng.standard_normal(512)).astype(f32)
    qx, sx = O.quant_rows(O.layer_norm(x1, la, lb))
    if scale_spread:   # row scales from 1e-35 to 1e25: the clamp, tiny and huge hidden rows
        sx = (sx * np.float32(10.0) ** rng.integers(-33, 26, M)).astype(f32)
    qw1, sw1 = O.quant_weight((rng.standard_normal((F, 512)) * 0.05).astype(f32), 8)
    qw2, sw2 = O.quant_weight((rng.standard_normal((512, F)) * 0.05).astype(f32), 8)
    b1 = (rng.standard_normal(F) * 0.1).astype(f32)
    b2 = (rng.standard_normal(512) * 0.1).astype(f32)
    na = (1 + 0.1 * rng.standard_normal(512)).astype(f32)
    nb = (0.1 * rng.standard_normal(512)).astype(f32)
    wf = torch.empty(F * 1024, dtype=torch.int8, device="cuda")
    assert lib().qtx_pack_ffn(P(dev(torch, qw1).data_ptr()), P(dev(torch, qw2).data_ptr()), F,
                              P(wf.data_ptr()), S0) == 0
    A = dev(torch, to_kp(qx))
    sa = dev(torch, sx)
    x = dev(torch, x1.copy())
    a = FfnRows()
    a.A, a.sa, a.wf = A.data_ptr(), sa.data_ptr(), wf.data_ptr()
    a.sw1, a.b1 = dev(torch, sw1).data_ptr(), dev(torch, b1).data_ptr()
    a.sw2, a.b2 = dev(torch, sw2).data_ptr(), dev(torch, b2).data_ptr()
    a.x, a.ln_a, a.ln_b = x.data_ptr(), dev(torch, na).data_ptr(), dev(torch, nb).data_ptr()
    a.M, a.F = M, F
    if lnq:
        q8 = A if alias else torch.zeros((M + (M & 1), 512), dtype=torch.int8, device="cuda")
        qs = sa if alias else torch.empty(M, dtype=torch.float32, device="cuda")
        a.lnq, a.lns = q8.data_ptr(), qs.data_ptr()
    else:
        lo = torch.empty((M, 512), dtype=torch.float32, device="cuda")
        a.lnout = lo.data_ptr()
    rc = lib().qtx_ffn_rows(C.byref(a), S0)
    assert rc == 0, lib().qtx_last_error()
    torch.cuda.synchronize()
    h = O.linear_epilogue(O.int_gemm(qx, qw1), sx, sw1, b1, relu=True)
    qh, sh = O.quant_rows(h)
    x2 = x1 + O.linear_epilogue(O.int_gemm(qh, qw2), sh, sw2, b2)
    np.testing.assert_array_equal(x.cpu().numpy(), x2)
    ln = O.layer_norm(x2, na, nb)
    if lnq:
        q, s = O.quant_rows(ln)
        np.testing.assert_array_equal(from_kp(q8.cpu().numpy(), M), q)
        np.testing.assert_array_equal(qs.cpu().numpy(), s)
    else:
        np.testing.assert_array_equal(lo.cpu().numpy(), ln)


@pytest.mark.parametrize("M,F,lnq", [(128, 2048, True), (300, 2048, True), (7, 2048, True),
                                     (4096, 2048, True), (300, 2048, False), (256, 1024, True),
                                     (129, 256, False)])
def test_ffn_rows(torch, M, F, lnq):
    """Full and ragged row blocks (M = 7 / 129 / 300), the fp32 final-norm output, and
    d_ff 1024 / 256 (16 / 4 chunks: the ring's short streams)."""
    ffn_case(torch, M, F, lnq)


def test_ffn_rows_scale_spread(torch):
    """Row scales from 1e-35 to 1e25: hidden rows from all-bias (the 1e-5 clamp of the
    hidden's scale) to ~1e24, through every quantizer and the LayerNorm's range guards."""
    ffn_case(torch, 1000, 2048, True, scale_spread=True)


def test_ffn_rows_in_place(torch):
    """lnq / lns aliasing A / sa, as the encoder calls it (each block reads its rows first)."""
    ffn_case(torch, 2048, 2048, True, alias=True, seed=5)


def test_ffn_rows_cfg3(torch):
    """cfg3's M = 32768 (256 blocks: one per CU), in place."""
    ffn_case(torch, 32768, 2048, True, alias=True, seed=9)
