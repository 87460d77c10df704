"""A/B of Q/K/V and FFN1 on k_gemm_wsq32 / k_gemm_wsy32 (QTX_WS32=1) against k_gemm_wsq / wsy, alternated in ONE process:
the QKV and FFN1 launches alone at cfg3's M (bench.time_row_gemms) and the whole cfg3 encoder.

    QTX_LIB_PATH=onnx-transformer_amd/qtx/libqtx_diag.so python tools/ws32_ab.py [rounds] [variants, e.g. 0,1,2]

(the 32x32x32 kernels are in the diagnostic library only).  Result (round 5): DESIGN.md §4.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "onnx-transformer_amd")]
import bench  # noqa: E402
from qtx import _lib  # noqa: E402
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import synthetic_state_dict  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    model = QtxModel(synthetic_state_dict(20241223))
    L = _lib.lib(build=False)
    vs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2"]
    res = {v: [] for v in vs}
    for r in range(rounds):
        for v in vs:
            os.environ["QTX_WS32"] = v
            L.qtx_debug_reload_knobs()
            g = bench.time_row_gemms(reps=20)
            enc = bench.time_encoder_cfg3(model) * 1e3
            d = {"qkv_us": round(g["qkv_quant"][0], 2), "ffn1_us": round(g["ffn1_quant_onepass"][0], 2),
                 "encoder_ms": round(enc, 4)}
            res[v].append(d)
            print(r, f"QTX_WS32={v}", json.dumps(d), flush=True)
    for v, runs in res.items():
        print("BEST", f"QTX_WS32={v}", json.dumps({k: min(x[k] for x in runs) for k in runs[0]}))


if __name__ == "__main__":
    main()
