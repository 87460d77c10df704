"""A/B of the cfg3 encoder QuantLinear launches (bench.time_row_gemms) and optionally the
whole cfg3 encoder across library builds, one child process per (build, round), alternated:

    python tools/lib_ab.py onnx-transformer_amd/qtx/libqtx.so onnx-transformer_amd/qtx/libqtx_diag.so [--rounds 2] [--enc] [--dec]

--dec adds ms per cfg2 greedy decode (B = 32, S = 72, 71 steps) and per B = 256 decode.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
sys.path[:0] = [%r, %r]
import bench
g = bench.time_row_gemms(reps=20)
out = {k: round(t, 2) for k, (t, _) in g.items()}
model = None
if %r or %r:
    from qtx.model import QtxModel
    from qtx.weights import synthetic_state_dict
    model = QtxModel(synthetic_state_dict(20241223))
if %r:
    out["encoder_ms"] = round(bench.time_encoder_cfg3(model) * 1e3, 4)
if %r:
    out["dec32_ms"] = round(bench.time_decode(model, 32, 72, 72, steps=5) * 1e3, 3)
    out["dec256_ms"] = round(bench.time_decode(model, 256, 72, 72, steps=3) * 1e3, 3)
print("RESULT", json.dumps(out))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--enc", action="store_true")
    ap.add_argument("--dec", action="store_true")
    a = ap.parse_args()
    res = {l: [] for l in a.libs}
    code = CHILD % (REPO, os.path.join(REPO, "onnx-transformer_amd"), a.enc, a.dec, a.enc, a.dec)
    for r in range(a.rounds):
        for l in a.libs:
            env = dict(os.environ, QTX_LIB_PATH=os.path.abspath(l))
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT")]
            if p.returncode != 0 or not line:
                print(p.stdout[-2000:], p.stderr[-4000:])
                sys.exit(1)
            d = json.loads(line[0][7:])
            res[l].append(d)
            print(r, os.path.basename(l), json.dumps(d), flush=True)
    for l, runs in res.items():
        best = {k: min(x[k] for x in runs) for k in runs[0]}
        print("BEST", os.path.basename(l), json.dumps(best),
              "gemm_sum", round(sum(v for k, v in best.items() if not k.endswith("_ms")), 1))


if __name__ == "__main__":
    main()
