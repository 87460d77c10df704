"""Host enqueue time vs GPU time of one greedy decode (is the decode host-bound?).

    QTX_GRAPH_STEPS=k python tools/host_probe.py
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "onnx-transformer_amd")
from bench import make_src  # noqa: E402
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402

B, S, L = 32, 72, 72
model = QtxModel(synthetic_state_dict(20241223), ModelConfig())
src, _ = make_src(np.random.default_rng(1000), B, S)
srcd = torch.from_numpy(src).cuda()
maskd = (srcd != 2).to(torch.uint8)
ids = torch.empty((B, L), dtype=torch.int64, device="cuda")
t0 = time.perf_counter()
model.greedy(srcd, maskd, max_len=L, start=0, out=ids)
torch.cuda.synchronize()
print(f"first call (capture + instantiate + run) {(time.perf_counter() - t0) * 1e3:.1f} ms")
for _ in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.greedy(srcd, maskd, max_len=L, start=0, out=ids)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {(t1 - t0) * 1e3:.2f} ms, total {(t2 - t0) * 1e3:.2f} ms")
