"""In-kernel phase cycles of the KP row GEMM with the residual + LayerNorm epilogue
(k_gemm_row<RE_RES_LN, FULL, -, KP>) at the cfg3 encoder's M, from s_memtime stamps
(diagnostic build, -DQTX_STAMPS): main loop, y, first staged half, the first group's
residual add / x store / LayerNorm / quant+store, the remaining groups — median over
workgroups, plus the spread of start and end times over the grid.
    python tools/stamp_bench.py build   (here: the diagnostic library)
    python tools/row_stamps.py          (GPU box)"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "onnx-transformer_amd")]
STAMP_LIB = os.path.join(REPO, "onnx-transformer_amd/qtx/libqtx_stamps.so")


def main():
    import torch
    os.environ["QTX_LIB_PATH"] = STAMP_LIB
    from qtx import _lib
    _lib.lib(build=False)
    raw = C.CDLL(STAMP_LIB)
    buf = torch.zeros((4096, 16), dtype=torch.int64, device="cuda")
    raw.qtx_debug_set_stamps_gemm(C.c_void_p(buf.data_ptr()))
    M, D, F = int(os.environ.get("QTX_STAMP_M", "32768")), 512, 2048
    rng = np.random.default_rng(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    sa = torch.full((M,), 0.01, device="cuda")
    sw = torch.full((F,), 0.01, device="cuda")
    bias = torch.zeros(F, device="cuda")
    out8 = torch.empty((M * F,), dtype=torch.int8, device="cuda")
    os_ = torch.empty((4 * M,), device="cuda")
    x = torch.randn((M, D), device="cuda")
    lna, lnb = torch.ones(D, device="cuda"), torch.zeros(D, device="cuda")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    names = ["main loop", "y", "stage half 0", "grp0 add+res issue", "grp0 x store", "grp0 LN",
             "grp0 quant+store", "rest (3 groups)"]
    order = [0, 1, 3, 5, 6, 7, 8, 9, 2]
    for name, K in [("o_res_ln", D), ("ffn2_res_ln", F)]:
        a = T(rng.integers(-127, 128, (M, K)).astype(np.int8))
        w = T(rng.integers(-127, 128, (D, K)).astype(np.int8))
        wk = torch.empty_like(w)
        _lib.call("qtx_pack_w_kp", C.c_void_p(w.data_ptr()), D, K, C.c_void_p(wk.data_ptr()), st)
        args = _lib.RowGemm()
        for k, v in dict(A=a, sa=sa, W=wk, sw=sw, bias=bias, M=M, N=D, K=K, kp=1, epi=1, res=x, xout=x,
                         ln_a=lna, ln_b=lnb, lnq=out8, lns=os_).items():
            setattr(args, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
        for _ in range(3):
            buf.zero_()
            _lib.call("qtx_linear_rows", C.byref(args), st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        buf.zero_()
        e0.record()
        _lib.call("qtx_linear_rows", C.byref(args), st)
        e1.record()
        torch.cuda.synchronize()
        s = buf.cpu().numpy()[:M // 128].astype(np.int64)[:, order]
        d = np.diff(s, axis=1)
        med = np.median(d, 0).astype(int)
        t0 = s[:, 0].min()
        print(f"{name}: {e0.elapsed_time(e1) * 1e3:.1f} us (stamped build), {len(s)} WGs; median cycles: "
              + ", ".join(f"{n} {v}" for n, v in zip(names, med)), flush=True)
        print(f"   start spread {s[:, 0].max() - t0} cyc, main-loop end {np.percentile(s[:, 1] - t0, [5, 50, 95]).astype(int).tolist()}, "
              f"end {np.percentile(s[:, -1] - t0, [5, 50, 95]).astype(int).tolist()} cyc after the first start", flush=True)


if __name__ == "__main__":
    main()
