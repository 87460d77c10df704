"""Encoder time at the decode configs (cfg2: B=32, S=72; cfg5: B=256, S=72) through
QtxModel.encode, HIP events — the once-per-decode part of the greedy decode."""
import os
import sys

import torch

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "onnx-transformer_amd")]
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402

m = QtxModel(synthetic_state_dict(20241223), ModelConfig())
cfgs = [(int(b), 72) for b in sys.argv[1:]] or [(32, 72), (256, 72)]
for B, S in cfgs:
    x = torch.randn((B, S, 512), device="cuda")
    mk = torch.ones((B, S), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        m.encode(x, mk)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        m.encode(x, mk)
    e1.record()
    torch.cuda.synchronize()
    print(f"encoder B={B} S={S}: {e0.elapsed_time(e1) / 10:.3f} ms", flush=True)
