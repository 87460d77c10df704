#!/bin/bash
# Encoder attention (tools/attn_bench.py) with the HEAD library (libqtx_abold.so, see
# tools/ab.sh) and the working tree, alternated, then the cfg3 encoder both ways.
OLD=$GRAFT_REPO_ROOT/onnx-transformer_amd/qtx/libqtx_abold.so
NEW=$GRAFT_REPO_ROOT/onnx-transformer_amd/qtx/libqtx.so
for r in 1 2; do
  for L in $OLD $NEW; do
    echo "== $(basename $L)"
    QTX_LIB_PATH=$L timeout -k 10 100 python tools/attn_bench.py 2>&1 | grep "quant ctx" || exit 1
  done
done
for L in $OLD $NEW; do
  QTX_LIB_PATH=$L timeout -k 10 100 python tools/enc_bench.py 2>&1 | grep encoder || exit 1
done
