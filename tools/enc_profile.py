"""Run the cfg3 encoder (B=256, S=128) a few times — for rocprofv3 kernel stats / PMC passes."""
import os
import sys

import torch

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "onnx-transformer_amd")]
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402

m = QtxModel(synthetic_state_dict(20241223), ModelConfig())
x = torch.randn((256, 128, 512), device="cuda")
mk = torch.ones((256, 128), dtype=torch.uint8, device="cuda")
for _ in range(int(os.environ.get("QTX_ENC_REPS", "5"))):
    m.encode(x, mk)
torch.cuda.synchronize()
