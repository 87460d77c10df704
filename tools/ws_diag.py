"""Diagnostic (GPU box): where a weight-stationary Q/K/V kernel's outputs differ from the
oracle — per QTX_WSQ value, M: mismatch counts by output tile, row % 32, column // 64 (the
wave), the scales, over 3 repeated launches.
    python tools/ws_diag.py 2 300 [4096 ...]"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "onnx-transformer_amd"), os.path.join(REPO, "tests")]


def main():
    import torch
    from oracle import qtx_oracle as O
    from qtx._lib import RowGemm, lib
    from test_gpu_ops import _to_kp
    f32 = np.float32
    os.environ["QTX_WSQ"] = sys.argv[1]
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    for M in map(int, sys.argv[2:]):
        rng = np.random.default_rng(M)
        qx, sx = O.quant_rows(rng.standard_normal((M, 512)).astype(f32))
        qw, sw = O.quant_weight((rng.standard_normal((1536, 512)) * 0.05).astype(f32), 8)
        b = (rng.standard_normal(1536) * 1e-3).astype(f32)
        wk = torch.empty((1536, 512), dtype=torch.int8, device="cuda")
        W, A, SA, SW, B = T(qw), T(_to_kp(qx)), T(sx), T(sw), T(b)
        assert lib().qtx_pack_w_ws(C.c_void_p(W.data_ptr()), 1536, 512, C.c_void_p(wk.data_ptr()), None) == 0
        y = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b)
        ref = [O.quant_rows(y[:, 512 * t:512 * (t + 1)]) for t in range(3)]
        for rep in range(3):
            out8 = torch.zeros((3, M, 512), dtype=torch.int8, device="cuda")
            os_ = torch.zeros((3, M), dtype=torch.float32, device="cuda")
            a = RowGemm()
            for k, v in dict(A=A, sa=SA, W=wk, sw=SW, bias=B, M=M, N=1536, K=512, epi=0, out8=out8,
                             ldo8=512, o8_ts=M * 512, os=os_, os_ts=M, kp=2).items():
                setattr(a, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
            assert lib().qtx_linear_rows(C.byref(a), None) == 0
            torch.cuda.synchronize()
            o8, osc = out8.cpu().numpy(), os_.cpu().numpy()
            for t in range(3):
                bad = o8[t] != ref[t][0]
                sbad = osc[t] != ref[t][1]
                r, c = np.nonzero(bad)
                print(f"M={M} rep={rep} tile {t}: {bad.sum()} bad q, {sbad.sum()} bad scales "
                      f"(rows {np.nonzero(sbad)[0][:12].tolist()})", flush=True)
                if bad.sum():
                    print("   by row%32:", np.bincount(r % 32, minlength=32).tolist())
                    print("   by col//64:", np.bincount(c // 64, minlength=8).tolist())
                    print("   by col%64//16:", np.bincount(c % 64 // 16, minlength=4).tolist(),
                          " by row block:", np.bincount(r // 32).tolist())
                    rr = r[0]
                    print("   first bad row", rr, "got", o8[t][rr, :16].tolist(), "want", ref[t][0][rr, :16].tolist())


if __name__ == "__main__":
    main()
