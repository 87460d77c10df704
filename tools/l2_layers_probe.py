"""Does L2 residency of the decode step's weights matter?  Per-step time of the cfg2 greedy
decode (B = 32, 71 steps) for models of 1, 2, 3 and 6 decoder+encoder layers: with 1-2
layers a step's int8 weights (≈ 4.2 MB per decoder layer, spread over the 8 XCDs'
4 MiB L2s) stay L2-resident from one step to the next, with 6 they cannot.  If the per-layer
increment of the step time is the same below and above that size, the step's kernels are
not waiting on the Infinity Cache for their weights.     python tools/l2_layers_probe.py"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "onnx-transformer_amd")]
import bench  # noqa: E402
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402

res = {}
for nl in (1, 2, 3, 6):
    cfg = ModelConfig(n_layers=nl)
    m = QtxModel(synthetic_state_dict(20241223, cfg), cfg)
    t71 = min(bench.time_decode(m, 32, 72, 72) for _ in range(3))
    t2 = min(bench.time_decode(m, 32, 72, 2) for _ in range(3))
    res[nl] = (t71 - t2) / 70 * 1e6
    print(f"layers {nl}: {res[nl]:.1f} us per step", flush=True)
    del m
ls = sorted(res)
for a, b in zip(ls, ls[1:]):
    print(f"  layers {a} -> {b}: {(res[b] - res[a]) / (b - a):.1f} us per added layer")
