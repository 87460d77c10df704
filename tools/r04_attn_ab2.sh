#!/bin/bash
# round 4: attention phase-order experiment libqtx_x3.so (QTX_EXP_ATTN_SWAP) — bit-exact
# tests on it, launch A/B against the product (alternated), then the stamped build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-attn_ab2}; mkdir -p $O
P=onnx-transformer_amd/qtx/libqtx.so; X=onnx-transformer_amd/qtx/libqtx_x3.so
QTX_LIB_PATH=$X timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or attention or encq or cfg3 or encode or encoder" > $O/pytest_x.log 2>&1; rc=$?
tail -2 $O/pytest_x.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for L in $P $X; do
    echo "== $(basename $L)" >> $O/ab.log
    QTX_LIB_PATH=$L timeout -k 10 100 python tools/attn_bench.py 2>&1 | grep "quant ctx" >> $O/ab.log || exit 1
  done
done
cat $O/ab.log
QTX_LIB_PATH=onnx-transformer_amd/qtx/libqtx_diag.so timeout -k 10 120 python tools/attn_stamps.py 2>&1 | grep -v amdgpu.ids | tee $O/attn_stamps.log
