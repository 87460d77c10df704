"""Run by tests/test_diag_build.py in a subprocess with QTX_LIB_PATH = libqtx_diag.so: every
measured-negative weight-stationary variant of the diagnostic build (csrc/diag/)
on one full and one ragged shape, bit-exact against the oracle — so the diagnostic sources
cannot drift from the product's numerics unnoticed.  Prints one line per case
and exits non-zero on the first mismatch."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "onnx-transformer_amd")]

import torch  # noqa: E402

from oracle import qtx_oracle as O  # noqa: E402
from qtx._lib import RowGemm, lib  # noqa: E402

f32 = np.float32
P = C.c_void_p
KEEP = []


def dev(a):
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    KEEP.append(t)
    return t


def to_kp(a):
    M, K = a.shape
    if M & 1:
        a = np.concatenate([a, np.zeros((1, K), a.dtype)])
    return np.ascontiguousarray(a.reshape(-1, 2, K // 64, 64).transpose(0, 2, 1, 3)).reshape(-1, K)


def from_kp(a, M):
    K = a.shape[1]
    return a.reshape(-1, K // 64, 2, 64).transpose(0, 2, 1, 3).reshape(-1, K)[:M]


def rows_call(**kw):
    a = RowGemm()
    for k, v in kw.items():
        setattr(a, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
    rc = lib().qtx_linear_rows(C.byref(a), P(0))
    assert rc == 0, lib().qtx_last_error()


def setenv(env):
    for k in ("QTX_WSQ", "QTX_WSY", "QTX_WS_PRIO", "QTX_WS_XG", "QTX_WSA2", "QTX_WSP_PMAX_SR5", "QTX_WS32"):
        os.environ.pop(k, None)
    os.environ.update(env)
    lib().qtx_debug_reload_knobs()


def ws32_pack_ref(w):
    """The WS32 order of k_gemm_wsq32 / wsy32 (csrc/diag/qtx_wsgemm_diag.hip), restated in
    numpy: 1 KB block ((t*8 + w)*16 + s)*2 + u, lane l (r = l & 31): W[512t + 64w + 32u +
    16((r >> 2) & 1) + 4(r >> 3) + (r & 3)][32s + 16(l >> 5) .. +16]."""
    N, K = w.shape
    t, wv, s, u, l = np.meshgrid(np.arange(N // 512), np.arange(8), np.arange(16), np.arange(2),
                                 np.arange(64), indexing="ij")
    r = l & 31
    n = 512 * t + 64 * wv + 32 * u + 16 * ((r >> 2) & 1) + 4 * (r >> 3) + (r & 3)
    k0 = 32 * s + 16 * (l >> 5)
    rows = w[n.reshape(-1)]
    idx = k0.reshape(-1)[:, None] + np.arange(16)[None, :]
    return np.take_along_axis(rows, idx, axis=1).reshape(N, K)


def operands(M, N, seed, ws32=False):
    rng = np.random.default_rng(seed)
    qx, sx = O.quant_rows(rng.standard_normal((M, 512)).astype(f32))
    # row scales from 1e-35 to 1e25: every magnitude of the shared-reciprocal division
    sx = (sx * np.float32(10.0) ** rng.integers(-33, 26, M)).astype(f32)
    qw, sw = O.quant_weight((rng.standard_normal((N, 512)) * 0.05).astype(f32), 8)
    b = (rng.standard_normal(N) * 1e-3).astype(f32)
    wk = torch.empty((N, 512), dtype=torch.int8, device="cuda")
    if ws32:
        assert lib().qtx_debug_pack_w_ws32(P(dev(qw).data_ptr()), N, 512, P(wk.data_ptr()), P(0)) == 0
        torch.cuda.synchronize()
        assert np.array_equal(wk.cpu().numpy(), ws32_pack_ref(qw)), "WS32 pack"
    else:
        assert lib().qtx_pack_w_ws(P(dev(qw).data_ptr()), N, 512, P(wk.data_ptr()), P(0)) == 0
    return qx, sx, qw, sw, b, wk


def qkv_case(M, kp=2):
    qx, sx, qw, sw, b, wk = operands(M, 1536, M + 5, ws32=kp == 4)
    out8 = torch.empty((3, M, 512), dtype=torch.int8, device="cuda")
    os_ = torch.empty((3, M), dtype=torch.float32, device="cuda")
    rows_call(A=dev(to_kp(qx)), sa=dev(sx), W=wk, sw=dev(sw), bias=dev(b), M=M, N=1536, K=512,
              epi=0, out8=out8, ldo8=512, o8_ts=M * 512, os=os_, os_ts=M, kp=kp)
    torch.cuda.synchronize()
    y = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b)
    for t in range(3):
        q, s = O.quant_rows(y[:, 512 * t:512 * (t + 1)])
        if not (np.array_equal(out8[t].cpu().numpy(), q) and np.array_equal(os_[t].cpu().numpy(), s)):
            return False
    return True


def ffn1_case(M, onepass, kp=3):
    qx, sx, qw, sw, b, wk = operands(M, 2048, M + 9, ws32=kp == 5)
    h8 = torch.zeros((M + (M & 1), 2048), dtype=torch.int8, device="cuda")
    sh = torch.full((M,), -1.0, dtype=torch.float32, device="cuda")
    base = dict(A=dev(to_kp(qx)), sa=dev(sx), W=wk, sw=dev(sw), bias=dev(b), M=M, N=2048, K=512)
    if onepass:
        gx = torch.zeros(((32 * M + 2048) // 4,), dtype=torch.float32, device="cuda")
        rows_call(**base, kp=kp, epi=3, pmax_out=gx, out8=h8, ldo8=2048, os=sh)
        nb = (M + 31) // 32
        if gx.view(torch.int32)[2 * (4 * 32 * nb) + 1].item() != 0:   # the exchange timed out
            return False
    else:
        pm = torch.empty((4, M), dtype=torch.float32, device="cuda")
        rows_call(**base, kp=2, epi=2, pmax_out=pm)
        rows_call(**base, kp=2, epi=3, pmax_in=pm, pmax_n=4, out8=h8, ldo8=2048, os=sh)
    torch.cuda.synchronize()
    h = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b, relu=True)
    qh, s = O.quant_rows(h)
    return np.array_equal(from_kp(h8.cpu().numpy(), M), qh) and np.array_equal(sh.cpu().numpy(), s)


CASES = [
    ("qkv k_gemm_wsp", {"QTX_WSQ": "0"}, qkv_case),
    ("qkv k_gemm_wss", {"QTX_WSQ": "2"}, qkv_case),
    ("qkv k_gemm_wsz", {"QTX_WSQ": "3"}, qkv_case),
    ("qkv k_gemm_wsa", {"QTX_WSQ": "4"}, qkv_case),
    ("qkv k_gemm_wsq prio", {"QTX_WS_PRIO": "1"}, qkv_case),
    ("qkv k_gemm_wsq no-XG", {"QTX_WS_XG": "0"}, qkv_case),
    ("ffn1 one-pass k_gemm_wsx", {"QTX_WSY": "0"}, lambda M: ffn1_case(M, True)),
    ("ffn1 two-pass k_gemm_wsa2", {"QTX_WSA2": "1"}, lambda M: ffn1_case(M, False)),
    ("ffn1 two-pass wsp pmax sr5", {"QTX_WSP_PMAX_SR5": "1"}, lambda M: ffn1_case(M, False)),
    ("qkv k_gemm_wsq32", {"QTX_WS32": "1"}, lambda M: qkv_case(M, 4)),
    ("qkv k_gemm_wsq32 SR16", {"QTX_WS32": "2"}, lambda M: qkv_case(M, 4)),
    ("ffn1 one-pass k_gemm_wsy32", {"QTX_WS32": "1"}, lambda M: ffn1_case(M, True, 5)),
]


def main():
    assert "diag" in os.environ.get("QTX_LIB_PATH", ""), "run with QTX_LIB_PATH=libqtx_diag.so"
    bad = 0
    for name, env, fn in CASES:
        setenv(env)
        for M in (4096, 300, 33):
            ok = fn(M)
            print(f"{name:28s} M={M:5d}: {'bit-exact' if ok else 'MISMATCH'}", flush=True)
            bad += not ok
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
