#!/bin/bash
# round 4: encoder attention experiment (diag build) — bit-exact tests on it, then the
# cfg3 attention launch A/B against the product library, alternated, then the encoder
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-attn_ab}; mkdir -p $O
P=onnx-transformer_amd/qtx/libqtx.so; D=onnx-transformer_amd/qtx/libqtx_diag.so
QTX_LIB_PATH=$D timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or attention or encq or cfg3 or encode or encoder" > $O/pytest_diag.log 2>&1; rc=$?
tail -3 $O/pytest_diag.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for L in $P $D; do
    echo "== $(basename $L)" >> $O/ab.log
    QTX_LIB_PATH=$L timeout -k 10 100 python tools/attn_bench.py >> $O/ab.log 2>&1 || exit 1
  done
done
cat $O/ab.log
for L in $P $D; do
  QTX_LIB_PATH=$L timeout -k 10 200 python tools/enc_bench.py 2>&1 | grep -i encoder | sed "s|^|$(basename $L) |" || exit 1
done
timeout -k 10 120 python tools/mall_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/mall_probe.log || exit 1
