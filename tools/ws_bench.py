"""A/B of the cfg3 QuantLinear launches: KP row GEMM (kp=1) vs weight-stationary (kp=2)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "onnx-transformer_amd")]
import bench  # noqa: E402

PEAK = 256 * 4096 * 2 * 2.4e9
for ws in (False, True, False, True):
    r = bench.time_row_gemms(ws=ws)
    tot = sum(v[0] for v in r.values())
    ops = sum(v[1] for v in r.values())
    print(("ws " if ws else "kp ") + " ".join(f"{k}={v[0]:.1f}us({v[1] / v[0] / 1e-6 / PEAK * 100:.0f}%)"
                                          for k, v in r.items()),
          f"total={tot:.1f}us frac={ops / tot / 1e-6 / PEAK:.3f}", flush=True)
