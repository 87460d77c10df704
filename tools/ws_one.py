"""Run one cfg3 QuantLinear launch (weight-stationary kernel) a few times, for rocprofv3
PMC passes:  python tools/ws_one.py {qkv|o|ffn1max|ffn1q} [reps]"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "onnx-transformer_amd")]


def main():
    import torch
    from qtx import _lib
    _lib.lib(build=False)
    which = sys.argv[1] if len(sys.argv) > 1 else "qkv"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    M, D, F = 32768, 512, 2048
    rng = np.random.default_rng(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    a = T(rng.integers(-127, 128, (M, D)).astype(np.int8))
    sa = torch.full((M,), 0.01, device="cuda")
    sw = torch.full((F,), 0.01, device="cuda")
    bias = torch.zeros(F, device="cuda")
    out8 = torch.empty((M * F + F,), dtype=torch.int8, device="cuda")
    os_ = torch.empty((4 * M,), device="cuda")
    x = torch.randn((M, D), device="cuda")
    lna, lnb = torch.ones(D, device="cuda"), torch.zeros(D, device="cuda")
    pm = torch.full((4, M), 3.0, device="cuda")
    N, kw = {"qkv": (3 * D, dict(epi=0, out8=out8, ldo8=D, o8_ts=M * D, os=os_, os_ts=M)),
             "o": (D, dict(epi=1, res=x, xout=x, ln_a=lna, ln_b=lnb, lnq=out8, lns=os_)),
             "ffn1max": (F, dict(epi=2, pmax_out=pm)),
             "ffn1q": (F, dict(epi=3, pmax_in=pm, pmax_n=4, out8=out8, ldo8=F, os=os_))}[which]
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    w = T(rng.integers(-127, 128, (N, D)).astype(np.int8))
    wk = torch.empty_like(w)
    _lib.call("qtx_pack_w_ws", C.c_void_p(w.data_ptr()), N, D, C.c_void_p(wk.data_ptr()), st)
    args = _lib.RowGemm()
    for k, v in dict(A=a, sa=sa, W=wk, sw=sw, bias=bias, M=M, N=N, K=D, kp=2, **kw).items():
        setattr(args, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
    for _ in range(reps):
        _lib.call("qtx_linear_rows", C.byref(args), st)
    torch.cuda.synchronize()
    print("ok", which, flush=True)


if __name__ == "__main__":
    main()
