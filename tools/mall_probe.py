"""Does the residual + LayerNorm epilogue of O / FFN2 (k_gemm_row<RE_RES_LN>, cfg3 M = 32768)
run faster when its residual rows are resident in the Infinity Cache?  Times each launch
alone (HIP events around it) in three cache states, interleaved:
  warm     the launch repeated back to back (what bench.time_row_gemms measures)
  cold     a 512 MiB buffer written before each launch (the residual comes from HBM)
  res      the same flush, then the residual rows read once (a torch sum) before the launch
Prints us per launch.   python tools/mall_probe.py"""
import ctypes as C
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "onnx-transformer_amd")]
import bench  # noqa: E402
from qtx import _lib  # noqa: E402

D, F, M = 512, 2048, 256 * 128
L = _lib.lib(build=False)
rng = np.random.default_rng(0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
a512 = T(bench._quantized_rows(rng, M, D))
a2048 = T(bench._quantized_rows(rng, M, F, relu=True))
sa = torch.full((M,), 0.01, device="cuda")
sw = torch.full((F,), 0.01, device="cuda")
bias = torch.zeros(F, device="cuda")
out8 = torch.empty((M * D,), dtype=torch.int8, device="cuda")
os_ = torch.empty((M,), device="cuda")
x = torch.randn((M, D), device="cuda")
lna, lnb = torch.ones(D, device="cuda"), torch.zeros(D, device="cuda")
flush = torch.empty((512 << 20) // 4, device="cuda")
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
cases = {}
for name, K, a in [("o_res_ln", D, a512), ("ffn2_res_ln", F, a2048)]:
    w = T(rng.integers(-127, 128, (D, K)).astype(np.int8))
    wk = torch.empty_like(w)
    _lib.call("qtx_pack_w_kp", C.c_void_p(w.data_ptr()), D, K, C.c_void_p(wk.data_ptr()), st)
    args = _lib.RowGemm()
    for k, v in dict(A=a, sa=sa, W=wk, sw=sw, bias=bias, M=M, N=D, K=K, kp=1, epi=1, res=x, xout=x,
                     ln_a=lna, ln_b=lnb, lnq=out8, lns=os_).items():
        setattr(args, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
    cases[name] = (args, wk)


def one(args, state):
    if state != "warm":
        flush.fill_(1.0)
    if state == "res":
        x.sum()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    L.qtx_linear_rows(C.byref(args), st)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3


for name, (args, _) in cases.items():
    for _ in range(3):
        one(args, "warm")
    t = {s: [] for s in ("warm", "cold", "res")}
    for r in range(10):
        for s in t:
            t[s].append(one(args, s))
    print(name, "  ".join(f"{s} {np.median(v):6.1f} us" for s, v in t.items()), flush=True)
