#!/bin/bash
# diagnostic libraries of k_skinny_wide with parts removed (QTX_ABL bitmask: 1 no weight
# loads, 2 no LayerNorm/quant chain, 4 no MFMA) -> onnx-transformer_amd/qtx/libqtx_abl<N>.so
cd $(dirname $0)/..; export PYTHONPATH=$PWD/onnx-transformer_amd
for n in "$@"; do
  python - <<PY
from qtx import _build
import shutil
p = _build.build(extra=["-DQTX_ABL=$n"])
shutil.move(p, "onnx-transformer_amd/qtx/libqtx_abl$n.so")
PY
done
