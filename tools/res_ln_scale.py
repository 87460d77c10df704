"""How the RES_LN row GEMMs (O, FFN2 on k_gemm_row<RE_RES_LN> KP) scale with M: one 128-row
tile per workgroup, so M = 32768 / 16384 / 8192 put 256 / 128 / 64 workgroups on the chip.
If the residual + LayerNorm epilogue is bound by the chip's HBM, half the workgroups take
about half its time; if it is bound per CU (bytes in flight), they take the same time.
usage: QTX_WS_RES_MAX_M=0 python tools/res_ln_scale.py"""
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "onnx-transformer_amd")]
os.environ.setdefault("QTX_WS_RES_MAX_M", "0")
import bench  # noqa: E402

for M in (32768, 16384, 8192):
    r = bench.time_row_gemms(M, reps=20)
    print(M, {k: round(t, 1) for k, (t, _) in r.items()}, flush=True)
