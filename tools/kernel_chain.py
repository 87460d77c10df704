"""In-graph cost of each decode-step kernel (the product step's amodes since round 6:
O / Oc and FFN2 quantize their fp32 input from its own rows, A_F32R): N back-to-back launches of one kernel captured
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


NLAYER = int(os.environ.get("QTX_CHAIN_LAYERS", "1"))   # distinct weight sets cycled (6: as the decode)


def chain_us(fn):
    for _ in range(3):
        fn(C.c_void_p(torch.cuda.current_stream().cuda_stream), 0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
            for i in range(N_LAUNCH):
                fn(st, i % NLAYER)
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
WL = [{nk: T(rng.integers(-127, 128, nk).astype(np.int8)) for nk in [(1536, 512), (512, 512), (2048, 512), (512, 2048)]}
      for _ in range(NLAYER)]
W = WL[0]
KVL = [(T(rng.integers(-127, 128, (B, 72, 512)).astype(np.int8)), T(rng.integers(-127, 128, (B, 72, 512)).astype(np.int8)))
       for _ in range(NLAYER)]
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
    return lambda st, l: _lib.call("qtx_skinny_linear", amode, Z, Z, P(X), ldx, P(lna), P(lnb), P(pin), pn,
                                   P(WL[l][(N, K)]), P(sw), P(bias), B, N, K, 8, flags, P(r), P(out), P(pout), st)


cases = {
    "LN+QKV   (A_LN, N=1536)": skinny(1, x, 512, None, 0, W[(1536, 512)], 1536, 512, 0),
    "self-attn (k_dec_attn, 41 keys)": lambda st, l: _lib.call(
        "qtx_decode_attention", 1, P(y), 1536, P(KVL[l][0]), P(KVL[l][1]), P(skc), P(svc), 72, P(step), 0, Z, B,
        P(ctx), P(pma), st),
    "O+res    (A_F32R, K=512)": skinny(3, ctx, 512, None, 0, W[(512, 512)], 512, 512, 2, res),
    "LN+Qc    (A_LN, N=512)": skinny(1, x, 512, None, 0, W[(512, 512)], 512, 512, 0),
    "cross-attn (72 keys)": lambda st, l: _lib.call(
        "qtx_decode_attention", 0, P(y), 512, P(KVL[l][0]), P(KVL[l][1]), P(skc), P(svc), 72, Z, 72, P(mask), B,
        P(ctx), P(pma), st),
    "LN+FFN1  (A_LN, N=2048, relu)": skinny(1, x, 512, None, 0, W[(2048, 512)], 2048, 512, 1),
    "FFN2+res (A_F32R, K=2048)": skinny(3, h, 2048, None, 0, W[(512, 2048)], 512, 2048, 2, res),
}
tot = 0.0
for name, fn in cases.items():
    t = chain_us(fn)
    tot += t
    print(f"B={B} {name:40s} {t:6.2f} us/launch", flush=True)
print(f"B={B} one decoder layer (8 launches, attention counted as listed): {tot + 0:.1f} us "
      f"(the cross-attn/O pair appears twice per layer: + {0:.1f})", flush=True)

# the 8 kernels of a decoder layer in the decode step's order, back to back (different code
# and data every launch, as in the real step) vs the sum of their single-kernel chains
order = ["LN+QKV   (A_LN, N=1536)", "self-attn (k_dec_attn, 41 keys)", "O+res    (A_F32R, K=512)",
         "LN+Qc    (A_LN, N=512)", "cross-attn (72 keys)", "O+res    (A_F32R, K=512)",
         "LN+FFN1  (A_LN, N=2048, relu)", "FFN2+res (A_F32R, K=2048)"]
fns = [cases[k] for k in order]


def layer_seq(st, l):
    for f in fns:
        f(st, l)


N_LAUNCH_SAVE = N_LAUNCH
N_LAUNCH = 12
t_layer = chain_us(layer_seq) * 1  # us per layer_seq call = per layer
print(f"B={B} decoder layer as the step's 8-kernel sequence: {t_layer:.1f} us "
      f"(sum of the single-kernel chains {tot + 2.6:.1f} us incl. the Oc twin)", flush=True)

# the step's tail: final LayerNorm + generator (k_generator_mfma, fp32 MFMA chain) and the
# log_softmax argmax + next embedding (k_argmax_embed), on the model's own weights
if os.environ.get("QTX_CHAIN_TAIL", "1") != "0":
    from qtx.model import QtxModel
    from qtx.weights import ModelConfig, synthetic_state_dict
    N_LAUNCH = N_LAUNCH_SAVE
    NLAYER = 1
    m = QtxModel(synthetic_state_dict(1), ModelConfig())
    V = 4444
    logits = torch.empty((B, V), device="cuda")
    ids = torch.zeros((B, 1300), dtype=torch.int64, device="cuda")
    stepd = torch.zeros(4, dtype=torch.int32, device="cuda")
    xn = torch.empty((B, 512), device="cuda")
    gids = torch.empty(B, dtype=torch.int64, device="cuda")
    gws = torch.empty(B * V, device="cuda")
    h = m.handle
    gen = lambda st, l: _lib.call("qtx_generator", h, P(x), B, P(logits), P(gids), P(gws), gws.numel() * 4, st)
    arg = lambda st, l: _lib.call("qtx_decode_argmax_embed", h, P(logits), B, P(ids), 1300, P(stepd), P(xn), st)
    print(f"B={B} {'generator + logsoftmax_argmax (2 kernels)':40s} {chain_us(gen):6.2f} us/launch", flush=True)
    stepd.zero_()
    print(f"B={B} {'argmax_embed (log_softmax argmax + embed)':40s} {chain_us(arg):6.2f} us/launch", flush=True)
    # the generator alone (QTX_STAMPS builds export it: QTX_LIB_PATH=.../libqtx_stamps.so)
    raw = C.CDLL(os.environ["QTX_LIB_PATH"]) if "stamps" in os.environ.get("QTX_LIB_PATH", "") else None
    if raw is not None:
        gwt = T((rng.standard_normal((4448, 512)) * 0.03).astype(np.float32))   # packed strips
        gb = T(np.zeros(V, np.float32))
        genm = lambda st, l: raw.qtx_debug_generator(P(x), B, P(lna), P(lnb), P(gwt), P(gb), V, P(logits), st)
        print(f"B={B} {'generator alone (k_generator_mfma, LN)':40s} {chain_us(genm):6.2f} us/launch", flush=True)
