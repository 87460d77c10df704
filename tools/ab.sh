#!/bin/bash
# A/B on one box: rows_bench + enc_bench with the committed-HEAD build ($GRAFT_REPO_ROOT/tools/ab_old.so)
# and the working-tree build, alternated twice.
KP=${KP:-0}
for r in 1 2; do
  for L in $GRAFT_REPO_ROOT/tools/ab_old.so $GRAFT_REPO_ROOT/onnx-transformer_amd/qtx/libqtx.so; do
    echo "== $L"
    QTX_BENCH_KP=$KP QTX_LIB_PATH=$L timeout -k 10 100 python tools/rows_bench.py 2>&1 | grep -v amdgpu || exit 1
    QTX_LIB_PATH=$L timeout -k 10 100 python tools/enc_bench.py 2>&1 | grep encoder || exit 1
  done
done
