"""Which live HIP-event measurement of the dominant decode kernel agrees with rocprofv3's
per-dispatch duration?  Runs the kernel (bench.run_dominant) four ways, in this order, and
prints the event-timed per-launch averages; run it under

    rocprofv3 --kernel-trace --stats -d gpurun_out/tp -o run -- python tools/dominant_timing_probe.py

and compare with tools/dispatch_runs.py gpurun_out/tp (per-run average durations).
  A eager, N back-to-back launches, one event pair
  B eager, one event pair per launch (synchronised), median
  C hipGraph of N launches, one event pair around the replay
  D hipGraph of N empty kernels (qtx_debug_nop)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "onnx-transformer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

B, N = 32, 256
one, keep = bench.run_dominant(B)
for i in range(8):
    one(i)
torch.cuda.synchronize()
ev = lambda: torch.cuda.Event(enable_timing=True)
# A
e0, e1 = ev(), ev()
e0.record()
for i in range(N):
    one(i)
e1.record()
torch.cuda.synchronize()
a = e0.elapsed_time(e1) * 1e3 / N
# B
ts = []
for i in range(N):
    e0, e1 = ev(), ev()
    e0.record()
    one(i)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
b = float(np.median(ts))
# C, D
c = bench.graph_time(lambda: [one(i) for i in range(N)]) / N
d = bench.graph_time(lambda: [bench.nop() for _ in range(N)]) / N
print({"eager_chain_us": a, "eager_single_median_us": b, "graph_chain_us": c, "graph_nop_us": d,
       "graph_minus_nop_us": c - d})
