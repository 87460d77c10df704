"""Per-phase in-kernel cycles of the weight-stationary GEMM (k_gemm_ws) from s_memtime
stamps: W load, then per row block the main loop and the epilogue (median over workgroups).
    python tools/ws_stamps.py build      (here: diagnostic library with -DQTX_STAMPS)
    python tools/ws_stamps.py            (GPU box)"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "onnx-transformer_amd")]
STAMP_LIB = os.path.join(REPO, "onnx-transformer_amd/qtx/libqtx_stamps.so")


def build():
    from qtx import _build
    cmd = [_build.hipcc(), *_build.FLAGS, "-DQTX_STAMPS", "-o", STAMP_LIB,
           *[os.path.join(_build.CSRC, s) for s in _build.SOURCES]]
    subprocess.run(cmd, check=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
        return
    import torch
    os.environ["QTX_LIB_PATH"] = STAMP_LIB
    from qtx import _lib
    L = _lib.lib(build=False)
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
    x = torch.randn((M, D), device="cuda")
    lna, lnb = torch.ones(D, device="cuda"), torch.zeros(D, device="cuda")
    pm = torch.full((4, M), 3.0, device="cuda")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, N, kw in [("qkv_quant", 3 * D, dict(epi=0, out8=out8, ldo8=D, o8_ts=M * D, os=os_, os_ts=M)),
                        ("o_res_ln", D, dict(epi=1, res=x, xout=x, ln_a=lna, ln_b=lnb, lnq=out8, lns=os_)),
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
        torch.cuda.synchronize()
        s = buf.cpu().numpy()
        nwg = 256 // (N // 512) * (N // 512)
        s = s[:nwg].astype(np.int64)
        t0 = s[:, 0]
        start = np.median(t0 - t0.min())
        wload = np.median(s[:, 1] - s[:, 0])
        phases = []
        prev = s[:, 1]
        for it in range(5):
            m_, e_ = s[:, 2 + 2 * it], s[:, 3 + 2 * it]
            ok = (m_ > 0) & (e_ > 0)
            if ok.sum() < nwg // 2:
                break
            phases.append((int(np.median((m_ - prev)[ok])), int(np.median((e_ - m_)[ok]))))
            prev = e_
        end = np.median(np.max(s[:, :12], axis=1) - t0)
        ex = s[:, 12:16]
        det = [int(np.median(ex[:, k] - s[:, 2])) if (ex[:, k] > 0).all() else None for k in range(4)]
        print(f"{name}: start skew {start:.0f}, W load + first DMA {wload:.0f}, per block (main, epi) "
              f"{phases}, total {end:.0f} cycles; block 0 after main: y {det[0]}, pre-barrier {det[1]}, "
              f"post-barrier {det[2]}, max done {det[3]}", flush=True)


if __name__ == "__main__":
    main()
