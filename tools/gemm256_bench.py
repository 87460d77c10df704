"""qtx_linear_i8 (k_gemm256: 256x256 tiles, BK=64, 4-stage ring, fp32 output) at the cfg3
QuantLinear shapes, for comparison with the row GEMM main loop."""
import ctypes as C
import os
import sys

import numpy as np
import torch

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
sys.path.insert(0, _R + "/onnx-transformer_amd")
from qtx import _lib  # noqa: E402

L = _lib.lib(build=False)
P = lambda t: C.c_void_p(t.data_ptr())
S0 = C.c_void_p(0)
M = 32768
for N, K in [(1536, 512), (512, 512), (2048, 512), (512, 2048)]:
    A = torch.randint(-127, 128, (M, K), dtype=torch.int8, device="cuda")
    W = torch.randint(-127, 128, (N, K), dtype=torch.int8, device="cuda")
    sa = torch.full((M,), 0.01, device="cuda")
    sw = torch.full((N,), 0.01, device="cuda")
    b = torch.zeros(N, device="cuda")
    out = torch.empty((M, N), device="cuda")
    f = lambda: L.qtx_linear_i8(P(A), P(sa), P(W), P(sw), P(b), M, N, K, 8, 0, S0, P(out), S0)
    for _ in range(3):
        assert f() == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        f()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10 * 1e3
    print(f"k_gemm256 N={N} K={K}: {t:.1f} us  {2 * M * N * K / t / 1e6 / 5033 * 100:.1f}% of int8 peak "
          f"(fp32 out {M * N * 4 / t / 1e6:.2f} TB/s)")
