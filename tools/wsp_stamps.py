"""Accumulated in-kernel phase cycles of the pipelined weight-stationary GEMM (k_gemm_wsp)
from s_memtime (diagnostic build, -DQTX_STAMPS): per workgroup the block-0 prologue, the
top-of-block wait (DMA + barrier), first half (MFMA + epilogue part 1), the mid barrier,
second half (MFMA + quantization) — median over workgroups.
    python tools/ws_stamps.py build      (here: diagnostic library with -DQTX_STAMPS)
    python tools/wsp_stamps.py           (GPU box)"""
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
    raw.qtx_debug_set_stamps_ws(C.c_void_p(buf.data_ptr()))
    M, D, F = 32768, 512, 2048
    rng = np.random.default_rng(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    a = T(rng.integers(-127, 128, (M, D)).astype(np.int8))
    sa = torch.full((M,), 0.01, device="cuda")
    sw = torch.full((F,), 0.01, device="cuda")
    bias = torch.zeros(F, device="cuda")
    out8 = torch.empty((M * F,), dtype=torch.int8, device="cuda")
    os_ = torch.empty((4 * M,), device="cuda")
    pm = torch.full((4, M), 3.0, device="cuda")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, N, kw in [("qkv_quant", 3 * D, dict(epi=0, out8=out8, ldo8=D, o8_ts=M * D, os=os_, os_ts=M)),
                        ("ffn1_rowmax", F, dict(epi=2, pmax_out=pm)),
                        ("ffn1_quant", F, dict(epi=3, pmax_in=pm, pmax_n=4, out8=out8, ldo8=F, os=os_))]:
        w = T(rng.integers(-127, 128, (N, D)).astype(np.int8))
        wk = torch.empty_like(w)
        _lib.call("qtx_pack_w_ws", C.c_void_p(w.data_ptr()), N, D, C.c_void_p(wk.data_ptr()), st)
        args = _lib.RowGemm()
        for k, v in dict(A=a, sa=sa, W=wk, sw=sw, bias=bias, M=M, N=N, K=D, kp=2, **kw).items():
            setattr(args, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
        for _ in range(3):
            buf.zero_()
            _lib.call("qtx_linear_rows", C.byref(args), st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("qtx_linear_rows", C.byref(args), st)
        e1.record()
        torch.cuda.synchronize()
        s = buf.cpu().numpy()[:256].astype(np.int64)
        s = s[s[:, 5] > 0]
        med = lambda c: int(np.median(s[:, c]))
        nb = med(6)
        print(f"{name}: {e0.elapsed_time(e1) * 1e3:.1f} us (stamped build), {len(s)} WGs x {nb} blocks; "
              f"median cycles: prologue+block0 {med(0)}, per block: top wait {med(1) / (nb - 1):.0f}, "
              f"half1 {med(2) / (nb - 1):.0f}, mid barrier {med(3) / (nb - 1):.0f}, half2 {med(4) / (nb - 1):.0f}; "
              f"total {med(5)}", flush=True)


if __name__ == "__main__":
    main()
