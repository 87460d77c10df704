"""cfg3 encoder attention (B=256, S=128): fp32-context kernel + quantization kernel vs the
fused quantized-context kernel (k_attn_encq).  Prints us per launch."""
import ctypes as C
import sys

import numpy as np
import torch

_R = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, _R)
sys.path.insert(0, _R + "/onnx-transformer_amd")
from qtx import _lib  # noqa: E402

L = _lib.lib(build=False)
B, S = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (256, 128)
rng = np.random.default_rng(0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
P = lambda t: C.c_void_p(t.data_ptr())
S0 = C.c_void_p(0)
q, k, v = (T(rng.integers(-127, 128, (B, S, 512)).astype(np.int8)) for _ in range(3))
sq, sk, sv = (T(rng.uniform(0.002, 0.03, (B, S)).astype(np.float32)) for _ in range(3))
km = T(np.ones((B, S), np.uint8))
ctx = torch.empty((B, S, 512), device="cuda")
ctx8 = torch.empty((B, S, 512), dtype=torch.int8, device="cuda")
sc = torch.empty((B, S), device="cuda")


def old():
    L.qtx_attention_i8(P(q), P(sq), P(k), P(sk), P(v), P(sv), P(km), S, 0, B, 8, S, S, P(ctx), 0, S0)


def new():
    L.qtx_attention_i8_quant(P(q), P(sq), P(k), P(sk), P(v), P(sv), P(km), B, S, P(ctx8), P(sc), S0)


for name, f in [("attn fp32 ctx", old), ("attn quant ctx", new)]:
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20 * 1e3
    flop = B * 8 * S * S * 64 * 2
    print(f"B={B} S={S} {name:16s} {t:8.1f} us  PV fp32 {flop / t / 1e6:6.1f} TFLOP/s")
