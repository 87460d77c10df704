"""Where the cfg2 decode time goes: encoder (B=32, S=72), cross K/V, steps (from totals)."""
import os
import sys
import time

import numpy as np
import torch

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R)
sys.path.insert(0, _R + "/onnx-transformer_amd")
import bench  # noqa: E402
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402

m = QtxModel(synthetic_state_dict(20241223), ModelConfig())
B, S = 32, 72
src, _ = bench.make_src(np.random.default_rng(1000), B, S)
srcd = torch.from_numpy(src).cuda()
mk = (srcd != 2).to(torch.uint8)
x = m.embed(srcd, "src")


def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


te = t(lambda: m.encode(x, mk))
for L in (2, 72):
    tg = t(lambda: m.greedy(srcd, mk, max_len=L), 10)
    print(f"greedy max_len={L}: {tg:.3f} ms")
print(f"encoder B={B} S={S}: {te:.3f} ms")
