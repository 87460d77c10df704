"""cfg3 encoder QuantLinear GEMM shapes (M = 256*128): time per GEMM and % of int8 peak.

    python tools/gemm_bench.py            (QTX_GEMM128=1 selects the old 128x128 kernel)
"""
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "onnx-transformer_amd")
from qtx import _lib  # noqa: E402

PEAK = 256 * 4096 * 2 * 2.4e9
M = 256 * 128
P = lambda t: C.c_void_p(t.data_ptr())
S0 = C.c_void_p(0)
L = _lib.lib()
rng = np.random.default_rng(0)
tot_t, tot_ops = 0.0, 0
for name, N, K, flags in [("QKV", 1536, 512, 0), ("O", 512, 512, 2), ("FFN1", 2048, 512, 1),
                          ("FFN2", 512, 2048, 2)]:
    a = torch.from_numpy(rng.integers(-127, 128, (M, K)).astype(np.int8)).cuda()
    w = torch.from_numpy(rng.integers(-127, 128, (N, K)).astype(np.int8)).cuda()
    sa, sw, b = torch.rand(M).cuda(), torch.rand(N).cuda(), torch.rand(N).cuda()
    out = torch.empty((M, N)).cuda()
    res = torch.rand((M, N)).cuda()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (P(a), P(sa), P(w), P(sw), P(b), M, N, K, 8, flags, P(res), P(out), st)
    for _ in range(3):
        L.qtx_linear_i8(*args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        L.qtx_linear_i8(*args)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / n
    ops = 2 * M * N * K
    tot_t += t
    tot_ops += ops
    print(f"{name:5s} N={N:5d} K={K:5d}: {t * 1e6:8.1f} us  {ops / t / 1e12:7.1f} TOPS  "
          f"{100 * ops / t / PEAK:5.1f} % of int8 peak")
print(f"layer total {tot_t * 1e6:.1f} us, {100 * tot_ops / tot_t / PEAK:.1f} % of peak; "
      f"x6 layers = {6 * tot_t * 1e6:.0f} us (north-star target <= 492 us)")
