"""cfg3 shapes (M = 256*128) through qtx_linear_rows, each epilogue mode: us and % of peak.
With QTX_LIB_PATH=<stamp lib> also prints per-phase cycles (main loop / epilogue)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

_R = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, _R)
sys.path.insert(0, _R + "/onnx-transformer_amd")
from qtx import _lib  # noqa: E402

PEAK = 256 * 4096 * 2 * 2.4e9
M = 256 * 128
KP = int(os.environ.get("QTX_BENCH_KP", "1"))
L = _lib.lib(build=not os.environ.get("QTX_LIB_PATH"))
stamps = None
if os.environ.get("QTX_LIB_PATH") and "stamps" in os.environ["QTX_LIB_PATH"]:
    stamps = torch.zeros((4096, 16), dtype=torch.int64, device="cuda")
    C.CDLL(os.environ["QTX_LIB_PATH"]).qtx_debug_set_stamps_gemm(C.c_void_p(stamps.data_ptr()))
rng = np.random.default_rng(0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
a512 = T(rng.integers(-127, 128, (M, 512)).astype(np.int8))
a2048 = T(rng.integers(-127, 128, (M, 2048)).astype(np.int8))
sa = torch.full((M,), 0.01, device="cuda")
W = {n_k: T(rng.integers(-127, 128, n_k).astype(np.int8)) for n_k in [(1536, 512), (512, 512), (2048, 512), (512, 2048)]}
sw = torch.full((2048,), 0.01, device="cuda")
bias = torch.zeros(2048, device="cuda")
out8 = torch.empty((M * 2048,), dtype=torch.int8, device="cuda")
os_ = torch.empty((4 * M,), device="cuda")
x = torch.randn((M, 512), device="cuda")
lna, lnb = torch.ones(512, device="cuda"), torch.zeros(512, device="cuda")
pm = torch.full((4, M), 3.0, device="cuda")
cases = [("QKV quant", 1536, 512, a512, dict(epi=0, out8=out8, ldo8=512, o8_ts=M * 512, os=os_, os_ts=M)),
         ("O res+LN", 512, 512, a512, dict(epi=1, res=x, xout=x, ln_a=lna, ln_b=lnb, lnq=out8, lns=os_)),
         ("FFN1 pmax", 2048, 512, a512, dict(epi=2, pmax_out=pm)),
         ("FFN1 quant", 2048, 512, a512, dict(epi=3, pmax_in=pm, pmax_n=4, out8=out8, ldo8=2048, os=os_)),
         ("FFN2 res+LN", 512, 2048, a2048, dict(epi=1, res=x, xout=x, ln_a=lna, ln_b=lnb, lnq=out8, lns=os_))]
tot = 0.0
for name, N, K, a, kw in cases:
    args = _lib.RowGemm()
    base = dict(A=a, sa=sa, W=W[(N, K)], sw=sw, bias=bias, M=M, N=N, K=K, **kw)
    if KP:     # the encoder's layout (random operands: only the weight order matters)
        wk = torch.empty_like(W[(N, K)])
        assert L.qtx_pack_w_kp(C.c_void_p(W[(N, K)].data_ptr()), N, K, C.c_void_p(wk.data_ptr()), None) == 0
        base.update(W=wk, kp=1)
    for k, v in base.items():
        setattr(args, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if stamps is not None:
        stamps.zero_()
    for _ in range(3):
        assert L.qtx_linear_rows(C.byref(args), st) == 0, L.qtx_last_error()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        L.qtx_linear_rows(C.byref(args), st)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / n
    tot += t
    ops = 2 * M * N * K
    extra = ""
    if stamps is not None:
        nblk = (N // 512) * (M // 128)
        s = stamps[:nblk, :16].cpu().numpy().astype(np.float64)
        if kw["epi"] == 1:
            d = np.median(np.diff(s[:, [0, 1, 3, 2]], axis=1), 0).astype(int).tolist()
            gq = np.median(np.diff(s[:, 5:10], axis=1), 0).astype(int).tolist()
            extra = f"  cyc (main loop, y, res+LN+quant) {d}; group 0 (v, xout, LN, quant+st) {gq}"
        else:
            d = np.median(np.diff(s[:, [0, 1, 3, 4, 2]], axis=1), 0).astype(int).tolist()
            extra = f"  cyc (main loop, y, row max, quant/store) {d}"
    print(f"{name:12s} {t * 1e6:7.1f} us  {100 * ops / t / PEAK:5.1f} % of int8 peak{extra}")
print(f"layer (5 launches) {tot * 1e6:.1f} us")
