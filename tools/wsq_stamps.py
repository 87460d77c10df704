"""Accumulated in-kernel phase cycles (s_memtime, diagnostic build -DQTX_STAMPS) of the
Q/K/V weight-stationary GEMMs at cfg3 (M = 32768): k_gemm_wsp (QTX_WSQ=0: prologue, top
wait, half 1, mid barrier, half 2) and k_gemm_wsq (QTX_WSQ=1: prologue, top wait, MFMA +
quantization, y) — medians over workgroups, per block.
    python tools/ws_stamps.py build      (here: the stamped library)
    python tools/wsq_stamps.py           (GPU box)"""
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
    M, D = 32768, 512
    rng = np.random.default_rng(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    a = T(rng.integers(-127, 128, (M, D)).astype(np.int8))
    sa = torch.full((M,), 0.01, device="cuda")
    sw = torch.full((3 * D,), 0.01, device="cuda")
    bias = torch.zeros(3 * D, device="cuda")
    out8 = torch.empty((M * 3 * D,), dtype=torch.int8, device="cuda")
    os_ = torch.empty((3 * M,), device="cuda")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    w = T(rng.integers(-127, 128, (3 * D, D)).astype(np.int8))
    wk = torch.empty_like(w)
    _lib.call("qtx_pack_w_ws", C.c_void_p(w.data_ptr()), 3 * D, D, C.c_void_p(wk.data_ptr()), st)
    args = _lib.RowGemm()
    for k, v in dict(A=a, sa=sa, W=wk, sw=sw, bias=bias, M=M, N=3 * D, K=D, kp=2, epi=0,
                     out8=out8, ldo8=D, o8_ts=M * D, os=os_, os_ts=M).items():
        setattr(args, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
    for wsq in sys.argv[1:] or ("0", "1"):
        os.environ["QTX_WSQ"] = wsq
        # >= 2 s of back-to-back launches first: the clock the chip holds under this load
        # (MI355X_MICROARCH.md, DVFS give-back item 6)
        for _ in range(3000):
            _lib.call("qtx_linear_rows", C.byref(args), st)
        buf.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.call("qtx_linear_rows", C.byref(args), st)
        e1.record()
        torch.cuda.synchronize()
        s = buf.cpu().numpy()[:256].astype(np.int64)
        s = s[s[:, 5] > 0]
        med = lambda c: float(np.median(s[:, c]))
        nb = med(6)
        per = lambda c: med(c) / max(nb - 1, 1)
        print(f"QTX_WSQ={wsq}: {e0.elapsed_time(e1) * 1e3:.1f} us (stamped), {len(s)} WGs x {nb:.0f} blocks; "
              f"median cycles: prologue+block0 {med(0):.0f}; per block: top wait {per(1):.0f}, "
              f"[wsp: half1 {per(2):.0f}, mid barrier {per(3):.0f}, half2 {per(4):.0f}] "
              f"[wsq: mfma+quant {per(2):.0f}, y {per(4):.0f}]; total {med(5):.0f}"
              + (f"; in-kernel clock {float(np.median(s[:, 5] / np.maximum(s[:, 7], 1))) * 100:.0f} MHz"
                 if wsq == "1" else ""), flush=True)
        if wsq == "1":      # absolute entry / exit on the 100 MHz clock (s_memrealtime)
            t0, t1 = s[:, 8], s[:, 9]
            print(f"   workgroup entry spread {(t0.max() - t0.min()) / 100:.2f} us, exit spread "
                  f"{(t1.max() - t1.min()) / 100:.2f} us, first entry to last exit "
                  f"{(t1.max() - t0.min()) / 100:.2f} us, median workgroup lifetime "
                  f"{np.median(t1 - t0) / 100:.2f} us", flush=True)
        if wsq == "1":      # per wave of WG 0..: top wait / MFMA+quant / y per block, median over WGs
            pw = buf.cpu().numpy().reshape(-1)[256 * 16:256 * 16 + 256 * 8 * 4].reshape(256, 8, 4).astype(np.int64)
            pw = pw[pw[:, 0, 3] > 1]
            per_w = np.median(pw[:, :, :3] / (pw[:, :, 3:4] - 1), axis=0)
            for w in range(8):
                print(f"   wave {w}: top wait {per_w[w, 0]:.0f}, mfma+quant {per_w[w, 1]:.0f}, y {per_w[w, 2]:.0f}")


def ffn1():
    """k_gemm_wsy (the one-pass FFN1, kp = 3) at cfg3: per-wave phase cycles per block."""
    import torch
    from qtx import _lib
    raw = C.CDLL(STAMP_LIB)
    buf = torch.zeros((4096, 16), dtype=torch.int64, device="cuda")
    raw.qtx_debug_set_stamps_ws(C.c_void_p(buf.data_ptr()))
    M, D, N = 32768, 512, 2048
    rng = np.random.default_rng(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    a = T(rng.integers(-127, 128, (M, D)).astype(np.int8))
    sa = torch.full((M,), 0.01, device="cuda")
    sw = torch.full((N,), 0.01, device="cuda")
    bias = torch.zeros(N, device="cuda")
    h8 = torch.empty((M, N), dtype=torch.int8, device="cuda")
    sh = torch.empty((M,), device="cuda")
    gx = torch.empty(((32 * M + 2048) // 4,), dtype=torch.float32, device="cuda")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    w = T(rng.integers(-127, 128, (N, D)).astype(np.int8))
    wk = torch.empty_like(w)
    _lib.call("qtx_pack_w_ws", C.c_void_p(w.data_ptr()), N, D, C.c_void_p(wk.data_ptr()), st)
    args = _lib.RowGemm()
    for k, v in dict(A=a, sa=sa, W=wk, sw=sw, bias=bias, M=M, N=N, K=D, kp=3, epi=3,
                     pmax_out=gx, out8=h8, ldo8=N, os=sh).items():
        setattr(args, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
    for _ in range(2000):
        _lib.call("qtx_linear_rows", C.byref(args), st)
    buf.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _lib.call("qtx_linear_rows", C.byref(args), st)
    e1.record()
    torch.cuda.synchronize()
    s = buf.cpu().numpy()[:256].astype(np.int64)
    s = s[s[:, 5] > 0]
    nb = float(np.median(s[:, 6]))
    print(f"FFN1 k_gemm_wsy: {e0.elapsed_time(e1) * 1e3:.1f} us (stamped), {len(s)} WGs x {nb:.0f} blocks, "
          f"median total {np.median(s[:, 5]):.0f} cycles ({np.median(s[:, 5]) / nb:.0f} per block)")
    pw = buf.cpu().numpy().reshape(-1)[256 * 16:256 * 16 + 256 * 8 * 8].reshape(256, 8, 8).astype(np.int64)
    pw = pw[pw[:, 0, 4] > 2]
    per_w = np.median(pw[:, :, :4] / (pw[:, :, 4:5] - 2), axis=0)
    for w in range(8):
        print(f"   wave {w}: top wait {per_w[w, 0]:.0f}, partner maxima {per_w[w, 1]:.0f}, "
              f"mfma+quant {per_w[w, 2]:.0f}, y {per_w[w, 3]:.0f}")


if __name__ == "__main__":
    if sys.argv[1:2] == ["ffn1"]:
        os.environ["QTX_LIB_PATH"] = STAMP_LIB
        ffn1()
        sys.exit(0)
    main()
