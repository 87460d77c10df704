"""In-graph cost of each decode-step kernel: N back-to-back launches of one kernel captured
in a hipGraph (torch.cuda.graph) and replayed — us per launch, to compare with the
dependent-kernel floor of tools/chain_probe.hip (same stream: every launch waits for the
previous one, as in the decode step)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "onnx-transformer_amd")]
from qtx import _lib  # noqa: E402

L = _lib.lib(build=False)
P = lambda t: C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)
rng = np.random.default_rng(0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
B = int(os.environ.get("QTX_CHAIN_B", "32"))
N_LAUNCH = 50


def chain_us(fn):
    for _ in range(3):
        fn(C.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
            for _ in range(N_LAUNCH):
                fn(st)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps / N_LAUNCH


y = T(rng.standard_normal((B, 1536)).astype(np.float32))
kc = T(rng.integers(-127, 128, (B, 72, 512)).astype(np.int8))
vc = T(rng.integers(-127, 128, (B, 72, 512)).astype(np.int8))
skc = T(np.full((B, 72), 0.01, np.float32))
svc = T(np.full((B, 72), 0.01, np.float32))
step = T(np.array([40, 0, 0, 0], np.int32))
mask = T(np.ones((B, 72), np.uint8))
x = T(rng.standard_normal((B, 512)).astype(np.float32))
h = T(np.abs(rng.standard_normal((B, 2048))).astype(np.float32))
W = {nk: T(rng.integers(-127, 128, nk).astype(np.int8)) for nk in [(1536, 512), (512, 512), (2048, 512), (512, 2048)]}
sw = T(np.full(2048, 0.01, np.float32))
bias = T(np.zeros(2048, np.float32))
out = torch.empty((B, 2048), device="cuda")
res = torch.empty((B, 512), device="cuda")
lna, lnb = T(np.ones(512, np.float32)), T(np.zeros(512, np.float32))
ctx = torch.empty((B, 512), device="cuda")
pma = T(np.full((8, B), 3.0, np.float32))
pmf = T(np.full((128, B), 3.0, np.float32))
pm_out = torch.empty((128, B), device="cuda")
Z = C.c_void_p(0)


def skinny(amode, X, ldx, pin, pn, w, N, K, flags, r=None, pout=None):
    return lambda st: _lib.call("qtx_skinny_linear", amode, Z, Z, P(X), ldx, P(lna), P(lnb), P(pin), pn,
                                P(w), P(sw), P(bias), B, N, K, 8, flags, P(r), P(out), P(pout), st)


cases = {
    "LN+QKV   (A_LN, N=1536)": skinny(1, x, 512, None, 0, W[(1536, 512)], 1536, 512, 0),
    "self-attn (k_dec_attn, 41 keys)": lambda st: _lib.call(
        "qtx_decode_attention", 1, P(y), 1536, P(kc), P(vc), P(skc), P(svc), 72, P(step), 0, Z, B,
        P(ctx), P(pma), st),
    "O+res    (A_F32Q, K=512)": skinny(2, ctx, 512, pma, 8, W[(512, 512)], 512, 512, 2, res),
    "LN+Qc    (A_LN, N=512)": skinny(1, x, 512, None, 0, W[(512, 512)], 512, 512, 0),
    "cross-attn (72 keys)": lambda st: _lib.call(
        "qtx_decode_attention", 0, P(y), 512, P(kc), P(vc), P(skc), P(svc), 72, Z, 72, P(mask), B,
        P(ctx), P(pma), st),
    "LN+FFN1  (A_LN, N=2048, relu+rowmax)": skinny(1, x, 512, None, 0, W[(2048, 512)], 2048, 512, 5, None, pm_out),
    "FFN2+res (A_F32Q, K=2048)": skinny(2, h, 2048, pmf, 128, W[(512, 2048)], 512, 2048, 2, res),
}
tot = 0.0
for name, fn in cases.items():
    t = chain_us(fn)
    tot += t
    print(f"B={B} {name:40s} {t:6.2f} us/launch", flush=True)
print(f"B={B} one decoder layer (8 launches, attention counted as listed): {tot + 0:.1f} us "
      f"(the cross-attn/O pair appears twice per layer: + {0:.1f})", flush=True)
