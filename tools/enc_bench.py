"""cfg3 encoder (B=256, S=128) ms per forward, through QtxModel.encode (HIP events)."""
import sys

import torch

_R = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, _R)
sys.path.insert(0, _R + "/onnx-transformer_amd")
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
m = QtxModel(synthetic_state_dict(20241223), ModelConfig())
x = torch.randn((B, 128, 512), device="cuda")
mk = torch.ones((B, 128), dtype=torch.uint8, device="cuda")
for _ in range(3):
    m.encode(x, mk)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    m.encode(x, mk)
e1.record()
torch.cuda.synchronize()
print(f"encoder B={B} S=128: {e0.elapsed_time(e1) / 10:.3f} ms")
