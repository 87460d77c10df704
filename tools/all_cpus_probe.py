"""How the CPU port behaves with torch.set_num_threads(os.cpu_count()) on the GPU box (the
whole host's CPUs, against the job's 16-CPU share): times a 2-sentence warm-up and 1, 2, 4
greedy steps of the cfg2 batch, printing each as it finishes.
    python tools/all_cpus_probe.py [threads]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "onnx-transformer_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else os.cpu_count()
torch.set_num_threads(n)
from bench import make_src  # noqa: E402
from oracle.torch_port import TorchPortModel  # noqa: E402
from qtx.weights import synthetic_state_dict  # noqa: E402

tp = TorchPortModel(synthetic_state_dict(20241223))
src, _ = make_src(np.random.default_rng(7), 32, 72)
m = torch.from_numpy((src != 2)[:, None, :])
s = torch.from_numpy(src)
t0 = time.perf_counter()
tp.greedy_decode(s[:2], m[:2], 4)
print(f"threads {n}: warm-up {time.perf_counter() - t0:.2f} s", flush=True)
for steps in (1, 2, 4):
    t0 = time.perf_counter()
    tp.greedy_decode(s, m, steps + 1)
    dt = time.perf_counter() - t0
    print(f"threads {n}: B=32, {steps} steps in {dt:.2f} s ({32 * steps / dt:.1f} tok/s)", flush=True)
