"""Greedy decodes of one batch, back to back, timed per decode (for the concurrency traces
of tools/conc_trace.sh: one process with QTX_DECODE_GROUPS sub-batch graphs, or two of these
processes at once).
    python tools/decode_conc.py --batch 256 --reps 6"""
import argparse
import os
import sys
import time

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "onnx-transformer_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--seed", type=int, default=1000)
    a = ap.parse_args()
    import torch
    import bench
    from qtx.model import QtxModel
    from qtx.weights import ModelConfig, synthetic_state_dict
    m = QtxModel(synthetic_state_dict(20241223), ModelConfig())
    src, _ = bench.make_src(np.random.default_rng(a.seed), a.batch, 72)
    srcd = torch.from_numpy(src).cuda()
    mk = (srcd != 2).to(torch.uint8)
    ids = torch.empty((a.batch, 72), dtype=torch.int64, device="cuda")
    for _ in range(2):
        m.greedy(srcd, mk, max_len=72, start=0, out=ids)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        m.greedy(srcd, mk, max_len=72, start=0, out=ids)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    h = ids.cpu().numpy().astype(np.int64)
    ck = int((h * (np.arange(h.size).reshape(h.shape) % 9973 + 1)).sum())
    print(f"pid {os.getpid()} B={a.batch} groups={os.environ.get('QTX_DECODE_GROUPS', '1')}: "
          f"ms per decode {['%.2f' % t for t in ts]} median {sorted(ts)[len(ts) // 2]:.2f} "
          f"ids checksum {ck}", flush=True)


if __name__ == "__main__":
    main()
