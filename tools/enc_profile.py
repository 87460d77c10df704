"""Run the cfg3 encoder (B=256, S=128) a few times — for rocprofv3 kernel stats."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "onnx-transformer_amd")
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402

m = QtxModel(synthetic_state_dict(20241223), ModelConfig())
x = torch.randn((256, 128, 512), device="cuda")
mk = torch.ones((256, 128), dtype=torch.uint8, device="cuda")
for _ in range(5):
    m.encode(x, mk)
torch.cuda.synchronize()
