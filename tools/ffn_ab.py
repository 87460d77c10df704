"""A/B of the encoder FFN at cfg3 in one process: the fused FFN launch (k_ffn_fused) against
the split launches (one-pass FFN1 + FFN2 row GEMM, the default; fused: QTX_FFN_FUSED_MIN_M=1), as whole cfg3
encoder forwards (HIP events, alternated rounds) and as the FFN launches alone.
    python tools/ffn_ab.py [rounds]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, _R + "/onnx-transformer_amd"]
from oracle import qtx_oracle as O  # noqa: E402
from qtx import _lib  # noqa: E402
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402

P = C.c_void_p


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def set_fused(on):
    if on:
        os.environ["QTX_FFN_FUSED_MIN_M"] = "1"
    else:
        os.environ.pop("QTX_FFN_FUSED_MIN_M", None)
    _lib.reload_knobs()


def launches(M=32768, F=2048):
    """The FFN launches alone on cfg3-shaped operands: fused vs one-pass FFN1 + FFN2."""
    lib = _lib.lib()
    rng = np.random.default_rng(1)
    x1 = (rng.standard_normal((M, 512)) * 2).astype(np.float32)
    qx, sx = O.quant_rows(x1)
    qw1, sw1 = O.quant_weight((rng.standard_normal((F, 512)) * 0.05).astype(np.float32), 8)
    qw2, sw2 = O.quant_weight((rng.standard_normal((512, F)) * 0.05).astype(np.float32), 8)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    kp = lambda a: np.ascontiguousarray(a.reshape(-1, 2, a.shape[1] // 64, 64).transpose(0, 2, 1, 3)).reshape(-1, a.shape[1])
    A, sa, w1, w2 = T(kp(qx)), T(sx), T(qw1), T(qw2)
    s1, b1, s2, b2 = T(sw1), T(rng.standard_normal(F).astype(np.float32) * 0.1), T(sw2), T(np.zeros(512, np.float32))
    la, lb = T(np.ones(512, np.float32)), T(np.zeros(512, np.float32))
    x = T(x1)
    wf = torch.empty(F * 1024, dtype=torch.int8, device="cuda")
    assert lib.qtx_pack_ffn(P(w1.data_ptr()), P(w2.data_ptr()), F, P(wf.data_ptr()), P(0)) == 0
    q8 = torch.empty((M, 512), dtype=torch.int8, device="cuda")
    qs = torch.empty(M, dtype=torch.float32, device="cuda")
    a = _lib.FfnRows()
    a.A, a.sa, a.wf, a.sw1, a.b1, a.sw2, a.b2 = (t.data_ptr() for t in (A, sa, wf, s1, b1, s2, b2))
    a.x, a.ln_a, a.ln_b, a.lnq, a.lns, a.M, a.F = x.data_ptr(), la.data_ptr(), lb.data_ptr(), q8.data_ptr(), qs.data_ptr(), M, F
    fused = lambda: lib.qtx_ffn_rows(C.byref(a), P(0))
    # the split launches: one-pass FFN1 (kp 3, WS weights) + FFN2 (kp 1, KP weights)
    w1ws = torch.empty((F, 512), dtype=torch.int8, device="cuda")
    w2kp = torch.empty((512, F), dtype=torch.int8, device="cuda")
    assert lib.qtx_pack_w_ws(P(w1.data_ptr()), F, 512, P(w1ws.data_ptr()), P(0)) == 0
    assert lib.qtx_pack_w_kp(P(w2.data_ptr()), 512, F, P(w2kp.data_ptr()), P(0)) == 0
    h8 = torch.empty((M, F), dtype=torch.int8, device="cuda")
    sh = torch.empty(M, dtype=torch.float32, device="cuda")
    gx = torch.zeros(((32 * M + 2048) // 4,), dtype=torch.float32, device="cuda")
    r1, r2 = _lib.RowGemm(), _lib.RowGemm()
    for r, kw in ((r1, dict(A=A, sa=sa, W=w1ws, sw=s1, bias=b1, M=M, N=F, K=512, kp=3, epi=3,
                            pmax_out=gx, out8=h8, ldo8=F, os=sh)),
                  (r2, dict(A=h8, sa=sh, W=w2kp, sw=s2, bias=b2, M=M, N=512, K=F, kp=1, epi=1,
                            res=x, xout=x, ln_a=la, ln_b=lb, lnq=q8, lns=qs))):
        for k, v in kw.items():
            setattr(r, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
    ffn1 = lambda: lib.qtx_linear_rows(C.byref(r1), P(0))
    ffn2 = lambda: lib.qtx_linear_rows(C.byref(r2), P(0))
    return fused, ffn1, ffn2


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    fused, ffn1, ffn2 = launches()
    for r in range(rounds):
        print(f"round {r}: fused FFN {timed(fused) * 1e3:.1f} us | split: FFN1 {timed(ffn1) * 1e3:.1f} us"
              f" + FFN2 {timed(ffn2) * 1e3:.1f} us", flush=True)
    m = QtxModel(synthetic_state_dict(20241223), ModelConfig())
    x = torch.randn((256, 128, 512), device="cuda")
    mk = torch.ones((256, 128), dtype=torch.uint8, device="cuda")
    for r in range(rounds):
        res = {}
        for on in (True, False):
            set_fused(on)
            res[on] = timed(lambda: m.encode(x, mk))
        print(f"round {r}: cfg3 encoder fused {res[True]:.3f} ms, split {res[False]:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
