"""A/B of the encoder QuantLinear launches (bench.time_row_gemms, cfg3 M = 32768) under
environment switches read at launch time, alternated in one process:

    python tools/gemm_ab.py QTX_WSQ=0 QTX_WSQ=1 [--reps 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "onnx-transformer_amd"))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+", help="NAME=VALUE[,NAME=VALUE] per variant")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    res = {c: [] for c in a.configs}
    for r in range(a.reps):
        for c in a.configs:
            for kv in c.split(","):
                k, v = kv.split("=")
                os.environ[k] = v
            g = bench.time_row_gemms(reps=10)
            res[c].append({k: round(t, 2) for k, (t, _) in g.items()})
            for kv in c.split(","):
                os.environ.pop(kv.split("=")[0])
    for c, runs in res.items():
        best = {k: min(r[k] for r in runs) for k in runs[0]}
        print(c, json.dumps(best), "sum", round(sum(best.values()), 1))


if __name__ == "__main__":
    main()
