"""Three cfg2 greedy decodes (B=32, S=72; QTX_PROF_B overrides B, e.g. 256 = cfg5's per-GPU
shard) — for rocprofv3 kernel stats of the decode alone."""
import os
import sys

import numpy as np
import torch

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "onnx-transformer_amd")]
import bench  # noqa: E402
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402

m = QtxModel(synthetic_state_dict(20241223), ModelConfig())
B = int(os.environ.get("QTX_PROF_B", "32"))
src, _ = bench.make_src(np.random.default_rng(1000), B, 72)
srcd = torch.from_numpy(src).cuda()
mk = (srcd != 2).to(torch.uint8)
ids = torch.empty((B, 72), dtype=torch.int64, device="cuda")
for _ in range(3):
    m.greedy(srcd, mk, max_len=72, start=0, out=ids)
torch.cuda.synchronize()
