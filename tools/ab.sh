#!/bin/bash
# A/B on one box: rows_bench + enc_bench with the committed-HEAD build
# (onnx-transformer_amd/qtx/libqtx_abold.so, built from `git archive HEAD`) and the
# working-tree build, alternated twice.
KP=${KP:-1}
OLD=$GRAFT_REPO_ROOT/onnx-transformer_amd/qtx/libqtx_abold.so
for r in 1 2; do
  for L in $OLD $GRAFT_REPO_ROOT/onnx-transformer_amd/qtx/libqtx.so; do
    echo "== $(basename $L)"
    QTX_BENCH_KP=$KP QTX_LIB_PATH=$L timeout -k 10 100 python tools/rows_bench.py 2>&1 | grep -v amdgpu || exit 1
    QTX_LIB_PATH=$L timeout -k 10 100 python tools/enc_bench.py 2>&1 | grep encoder || exit 1
  done
done
