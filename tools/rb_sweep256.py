"""Row-block sweep of the decode's skinny GEMMs at a large per-GPU batch (cfg5's shard,
B = 256), in one process on the diagnostic library (QTX_RB_* / QTX_SKINNY_WIDE are
diagnostic knobs), alternated over rounds; ids checked equal to the default's.

    python tools/rb_sweep256.py [B] [rounds]
"""
import os
import sys

import numpy as np
import torch

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "onnx-transformer_amd")]
os.environ.setdefault("QTX_LIB_PATH", os.path.join(_R, "onnx-transformer_amd/qtx/libqtx_diag.so"))
import bench  # noqa: E402
from qtx import _lib  # noqa: E402
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402

KNOBS = ("QTX_RB_I8_512", "QTX_RB_LN", "QTX_RB_I8_2048", "QTX_RB_F32Q", "QTX_SKINNY_WIDE",
         "QTX_FFN_QKERNEL", "QTX_SPLIT_LN", "QTX_ATTN_PM", "QTX_DEC_ATTN_GRP",
         "QTX_HQUANT_ROWS")
CONFIGS = [
    {},
    {"QTX_SKINNY_WIDE": "8"},
    {"QTX_SKINNY_WIDE": "8", "QTX_RB_F32Q": "8"},
    {"QTX_SKINNY_WIDE": "8", "QTX_RB_F32Q": "16"},
    {"QTX_SKINNY_WIDE": "8", "QTX_RB_F32Q": "32"},
    {"QTX_SKINNY_WIDE": "4"},
    {"QTX_SKINNY_WIDE": "4", "QTX_RB_F32Q": "16"},
    {"QTX_SKINNY_WIDE": "16", "QTX_RB_F32Q": "16"},
]
if os.environ.get("RB_SWEEP_SET") == "7":   # the hidden's quantization kernel
    CONFIGS = [{}, {"QTX_HQUANT_ROWS": "1"}]
if os.environ.get("RB_SWEEP_SET") == "6":   # every K = 512 GEMM N-split at small batches
    CONFIGS = [{}, {"QTX_SKINNY_WIDE": "4"}, {"QTX_SKINNY_WIDE": "8"}]
if os.environ.get("RB_SWEEP_SET") == "5":   # decode attention: one workgroup per sentence
    CONFIGS = [{}, {"QTX_DEC_ATTN_GRP": "0"}, {"QTX_DEC_ATTN_GRP": "1"}]
if os.environ.get("RB_SWEEP_SET") == "4":   # attention scales from partial maxima
    CONFIGS = [{}, {"QTX_ATTN_PM": "0"}, {"QTX_ATTN_PM": "1"}]
if os.environ.get("RB_SWEEP_SET") == "3":   # the hidden / LayerNorm done once per row
    CONFIGS = [
        {},
        {"QTX_FFN_QKERNEL": "1"},
        {"QTX_FFN_QKERNEL": "1", "QTX_RB_I8_2048": "16"},
        {"QTX_FFN_QKERNEL": "1", "QTX_RB_I8_2048": "32"},
        {"QTX_SPLIT_LN": "1"},
        {"QTX_SPLIT_LN": "1", "QTX_FFN_QKERNEL": "1", "QTX_RB_I8_2048": "16"},
        {"QTX_RB_F32Q": "32"},
        {"QTX_RB_F32Q": "8"},
    ]
if os.environ.get("RB_SWEEP_SET") == "1":   # the first sweep's single-knob set
    CONFIGS = [
        {},
        {"QTX_RB_F32Q": "16"},
        {"QTX_RB_F32Q": "32"},
        {"QTX_RB_I8_512": "16"},
        {"QTX_RB_I8_512": "32"},
        {"QTX_RB_LN": "8"},
        {"QTX_RB_LN": "16"},
        {"QTX_SKINNY_WIDE": "8"},
        {"QTX_SKINNY_WIDE": "16"},
        {"QTX_RB_F32Q": "16", "QTX_RB_I8_512": "16", "QTX_RB_LN": "16"},
    ]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    m = QtxModel(synthetic_state_dict(20241223), ModelConfig())
    src, _ = bench.make_src(np.random.default_rng(1000), B, 72)
    srcd = torch.from_numpy(src).cuda()
    mk = (srcd != 2).to(torch.uint8)
    ids = torch.empty((B, 72), dtype=torch.int64, device="cuda")
    ref = None
    res = {i: [] for i in range(len(CONFIGS))}
    for r in range(rounds):
        for i, cfg in enumerate(CONFIGS):
            for k in KNOBS:
                os.environ.pop(k, None)
            os.environ.update(cfg)
            _lib.reload_knobs()
            m.greedy(srcd, mk, max_len=72, start=0, out=ids)
            torch.cuda.synchronize()
            if ref is None:
                ref = ids.clone()
            ok = bool(torch.equal(ids, ref))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                m.greedy(srcd, mk, max_len=72, start=0, out=ids)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 3
            res[i].append(ms)
            print(f"round {r} {cfg or 'default'}: {ms:.3f} ms ids_equal={ok}", flush=True)
    for i, cfg in enumerate(CONFIGS):
        print(f"{str(cfg or 'default'):80s} {' '.join(f'{v:.3f}' for v in res[i])}")


if __name__ == "__main__":
    main()
