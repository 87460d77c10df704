"""Steady-state per-kernel latency of the decode kernels (graph-captured, back to back).

    python tools/kernel_bench.py [B]

Each kernel is called N times inside one torch CUDA graph; the replay is timed with
events, so the figure is launch gap + kernel critical path, as inside the decode graph.
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "onnx-transformer_amd")
from qtx import _lib  # noqa: E402

P = lambda t: C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)
S0 = C.c_void_p(0)


def timeit(fn, n=50, reps=10):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn(C.c_void_p(s.cuda_stream))
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn(C.c_void_p(s.cuda_stream))
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps / n


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    dev = "cuda"
    rng = np.random.default_rng(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    x = T(rng.standard_normal((B, 512)).astype(np.float32))
    h = T(np.abs(rng.standard_normal((B, 2048))).astype(np.float32))
    a8 = T(rng.integers(-127, 128, (B, 2048)).astype(np.int8))
    sa = T(np.full(B, 0.01, np.float32))
    q8 = torch.empty((B, 2048), dtype=torch.int8, device=dev)
    s8 = torch.empty(B, device=dev)
    lna, lnb = T(np.ones(512, np.float32)), T(np.zeros(512, np.float32))
    W = {(n, k): T(rng.integers(-127, 128, (n, k)).astype(np.int8)) for n, k in
         [(1536, 512), (512, 512), (2048, 512), (512, 2048)]}
    sw = T(np.full(2048, 0.01, np.float32))
    bias = T(np.zeros(2048, np.float32))
    out = torch.empty((B, 2048), device=dev)
    L = _lib.lib()
    res = {}

    res["row_quant 2048"] = timeit(lambda st: L.qtx_row_quant(P(h), B, 2048, 127.0, P(q8), P(s8), st))
    res["ln_quant 512"] = timeit(lambda st: L.qtx_layernorm_quant(P(x), P(lna), P(lnb), B, 512, S0, P(q8), P(s8), st))

    pmi = T(np.full((128, B), 3.0, np.float32))        # partial row maxima (A_F32Q)
    pmo = torch.empty((128, B), device=dev)

    def sk(amode, N, K, flags=0, nparts=128):
        return lambda st: L.qtx_skinny_linear(amode, P(a8), P(sa), P(x if K == 512 else h), K,
                                              P(lna), P(lnb), P(pmi), nparts, P(W[(N, K)]),
                                              P(sw), P(bias), B, N, K, 8, flags, P(out), P(out),
                                              P(pmo), st)
    res["skinny I8 512x512"] = timeit(sk(0, 512, 512))
    res["skinny I8 512x512 +res"] = timeit(sk(0, 512, 512, 2))
    res["skinny I8 1536x512"] = timeit(sk(0, 1536, 512))
    res["skinny I8 512x2048 +res"] = timeit(sk(0, 512, 2048, 2))
    res["skinny LN 1536x512"] = timeit(sk(1, 1536, 512))
    res["skinny LN 512x512"] = timeit(sk(1, 512, 512))
    res["skinny LN 2048x512 relu"] = timeit(sk(1, 2048, 512, 1))
    res["skinny F32Q 512x2048"] = timeit(sk(2, 512, 2048, 2))
    res["skinny F32Q 512x512 +res"] = timeit(sk(2, 512, 512, 2, 8))
    res["skinny LN 2048x512 relu+pmax"] = timeit(sk(1, 2048, 512, 5))

    y = T(rng.standard_normal((B, 1536)).astype(np.float32))
    kc = T(rng.integers(-127, 128, (B, 72, 512)).astype(np.int8))
    vc = T(rng.integers(-127, 128, (B, 72, 512)).astype(np.int8))
    skc = T(np.full((B, 72), 0.01, np.float32))
    svc = T(np.full((B, 72), 0.01, np.float32))
    step = T(np.array([40], np.int32))
    mask = T(np.ones((B, 72), np.uint8))
    ctx = torch.empty((B, 512), device=dev)
    pma = torch.empty((8, B), device=dev)
    res["dec attn self step40"] = timeit(lambda st: L.qtx_decode_attention(
        1, P(y), 1536, P(kc), P(vc), P(skc), P(svc), 72, P(step), 0, S0, B, P(ctx), P(pma), st))
    res["dec attn cross S72"] = timeit(lambda st: L.qtx_decode_attention(
        0, P(y), 512, P(kc), P(vc), P(skc), P(svc), 72, S0, 72, P(mask), B, P(ctx), P(pma), st))
    # generator (+ log_softmax/argmax) through a tiny model handle
    from qtx.model import QtxModel
    from qtx.weights import ModelConfig, synthetic_state_dict
    m = QtxModel(synthetic_state_dict(1, ModelConfig(n_layers=1)), ModelConfig(n_layers=1))
    logp = torch.empty((B, 4444), device=dev)
    ids = torch.empty(B, dtype=torch.int64, device=dev)
    wsg = torch.empty(B * 4444, device=dev)
    res["generator+lsm_argmax"] = timeit(lambda st: L.qtx_generator(
        m.handle, P(x), B, S0, P(ids), P(wsg), wsg.numel() * 4, st))
    for k, v in res.items():
        print(f"{k:28s} {v:7.2f} us")


if __name__ == "__main__":
    main()
