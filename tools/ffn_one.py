"""The fused FFN launch alone at cfg3 shapes, a few times (for rocprofv3 PMC passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ffn_ab  # noqa: E402

fused, ffn1, ffn2 = ffn_ab.launches()
which = sys.argv[1] if len(sys.argv) > 1 else "fused"
fn = {"fused": fused, "ffn1": ffn1, "ffn2": ffn2}[which]
for _ in range(5):
    fn()
torch.cuda.synchronize()
