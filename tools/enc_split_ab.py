"""A/B of the cfg3 encoder (B=256, S=128) with and without the two-stream sub-batch split
(QTX_ENC_NOSPLIT), interleaved rounds in one process."""
import os
import sys

import torch

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "onnx-transformer_amd")]
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import synthetic_state_dict  # noqa: E402

m = QtxModel(synthetic_state_dict(1))
x = torch.randn((256, 128, 512), device="cuda")
mk = torch.ones((256, 128), dtype=torch.uint8, device="cuda")


def t(n=5):
    for _ in range(2):
        m.encode(x, mk)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        m.encode(x, mk)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


res = {"split": [], "nosplit": []}
for r in range(3):
    for k in res:
        if k == "nosplit":
            os.environ["QTX_ENC_NOSPLIT"] = "1"
        else:
            os.environ.pop("QTX_ENC_NOSPLIT", None)
        res[k].append(t())
print({k: [round(v, 3) for v in vs] for k, vs in res.items()}, "ms per encoder")
