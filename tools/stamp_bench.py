"""Per-phase in-kernel timing of the decode kernels from s_memtime stamps.

Build the diagnostic library here (never shipped as the product):
    hipcc ... -DQTX_STAMPS -o onnx-transformer_amd/qtx/libqtx_stamps.so   (see main())
Run on the GPU box:
    QTX_LIB_PATH=onnx-transformer_amd/qtx/libqtx_stamps.so python tools/stamp_bench.py
Prints, per kernel, the median over workgroups of the cycles between consecutive stamps
(thread 0 of each block), and the spread of block start times.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "onnx-transformer_amd")
STAMP_LIB = "onnx-transformer_amd/qtx/libqtx_stamps.so"


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
    for unit in ("decode", "attn"):
        getattr(raw, f"qtx_debug_set_stamps_{unit}")(C.c_void_p(buf.data_ptr()))
    P = lambda t: C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)
    S0 = C.c_void_p(0)
    B = 32
    rng = np.random.default_rng(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    y = T(rng.standard_normal((B, 1536)).astype(np.float32))
    kc = T(rng.integers(-127, 128, (B, 72, 512)).astype(np.int8))
    vc = T(rng.integers(-127, 128, (B, 72, 512)).astype(np.int8))
    skc = T(np.full((B, 72), 0.01, np.float32))
    svc = T(np.full((B, 72), 0.01, np.float32))
    step = T(np.array([40], np.int32))
    mask = T(np.ones((B, 72), np.uint8))
    a8 = T(rng.integers(-127, 128, (B, 2048)).astype(np.int8))
    sa = T(np.full(B, 0.01, np.float32))
    x = T(rng.standard_normal((B, 512)).astype(np.float32))
    W = T(rng.integers(-127, 128, (1536, 512)).astype(np.int8))
    sw = T(np.full(2048, 0.01, np.float32))
    bias = T(np.zeros(2048, np.float32))
    out = torch.empty((B, 2048), device="cuda")
    lna, lnb = T(np.ones(512, np.float32)), T(np.zeros(512, np.float32))
    h = T(np.abs(rng.standard_normal((B, 2048))).astype(np.float32))
    W2 = T(rng.integers(-127, 128, (512, 2048)).astype(np.int8))
    ctx = torch.empty((B, 512), device="cuda")
    pma = torch.empty((8, B), device="cuda")
    pmi = T(np.full((128, B), 3.0, np.float32))
    gwt = T((rng.standard_normal((4448, 512)) * 0.03).astype(np.float32))   # packed strips
    gb = T(np.zeros(4444, np.float32))
    lg = torch.empty((B, 4444), device="cuda")
    L.qtx_generator_stamp = raw.qtx_debug_generator
    Be, Se = 256, 128                       # cfg3 encoder attention
    qe = T(rng.integers(-127, 128, (Be, Se, 512)).astype(np.int8))
    se = T(np.full((Be, Se), 0.01, np.float32))
    me = T(np.ones((Be, Se), np.uint8))
    ce = torch.empty((Be, Se, 512), device="cuda")
    cases = {
        "attn_mfma cfg3": (lambda: L.qtx_attention_i8(P(qe), P(se), P(qe), P(se), P(qe), P(se), P(me), Se, 0, Be, 8, Se, Se, P(ce), 0, S0), 8 * Be, 5),
        "dec_attn self": (lambda: L.qtx_decode_attention(1, P(y), 1536, P(kc), P(vc), P(skc), P(svc), 72, P(step), 0, S0, B, P(ctx), P(pma), S0), 8 * B, 5),
        "dec_attn cross": (lambda: L.qtx_decode_attention(0, P(y), 512, P(kc), P(vc), P(skc), P(svc), 72, S0, 72, P(mask), B, P(ctx), P(pma), S0), 8 * B, 5),
        "skinny I8 1536": (lambda: L.qtx_skinny_linear(0, P(a8), P(sa), S0, 512, S0, S0, S0, 0, P(W), P(sw), P(bias), B, 1536, 512, 8, 0, S0, P(out), S0, S0), 96 * B // 8, 4),
        "skinny LN 1536": (lambda: L.qtx_skinny_linear(1, S0, S0, P(x), 512, P(lna), P(lnb), S0, 0, P(W), P(sw), P(bias), B, 1536, 512, 8, 0, S0, P(out), S0, S0), 96 * B // 4, 4),
        "generator 32x4444": (lambda: L.qtx_generator_stamp(P(x), B, P(lna), P(lnb), P(gwt), P(gb), 4444, P(lg), S0), 72 * 2, 4),
        "skinny F32Q 512x2048": (lambda: L.qtx_skinny_linear(2, S0, S0, P(h), 2048, S0, S0, P(pmi), 128, P(W2), P(sw), P(bias), B, 512, 2048, 8, 2, P(out), P(out), S0, S0), 32 * B // 4, 4),
    }
    for name, (fn, nblk, nst) in cases.items():
        for _ in range(3):
            buf.zero_()
            fn()
            torch.cuda.synchronize()
        st = buf[:nblk, :nst].cpu().numpy().astype(np.float64)
        d = np.diff(st, axis=1)
        start_spread = st[:, 0].max() - st[:, 0].min()
        total = st[:, -1].max() - st[:, 0].min()
        print(f"{name:16s} phases(median cyc) {np.median(d, 0).astype(int).tolist()}  "
              f"block-start spread {start_spread:.0f}  first-start->last-end {total:.0f} cyc "
              f"({total / 2400:.2f} us)")

    # the decode tail: argmax_embed is the last kernel of every step, so after a greedy
    # decode its stamps (32 blocks, slots 0..5) are the ones left in the buffer
    from qtx.model import QtxModel
    from qtx.weights import ModelConfig, synthetic_state_dict
    m = QtxModel(synthetic_state_dict(1), ModelConfig())
    src = torch.full((B, 72), 2, dtype=torch.int64, device="cuda")
    src[:, :40] = 7
    src[:, 0] = 0
    src[:, 39] = 1
    mk = (src != 2).to(torch.uint8)
    for _ in range(2):
        buf.zero_()
        m.greedy(src, mk, max_len=72)
        torch.cuda.synchronize()
    st = buf[:B, :6].cpu().numpy().astype(np.float64)
    print(f"{'argmax_embed':16s} phases(median cyc) {np.median(np.diff(st, axis=1), 0).astype(int).tolist()}")


if __name__ == "__main__":
    main()

