#!/bin/bash
# round 4: k_attn_encv (VALU PV) in the product library — the attention / encoder GPU
# tests on it (bit-exact vs the oracle), then the cfg3 attention launch A/B against
# libqtx_x3.so (built with -DQTX_ATTN_ENCV=0: k_attn_encq<true>), alternated, then the encoder
# (the k_attn_encv experiment of profiles/r04_pv_valu.md; its source was reverted)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-encv_ab}; mkdir -p $O
P=onnx-transformer_amd/qtx/libqtx.so; X=onnx-transformer_amd/qtx/libqtx_x3.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_model.py tests/test_gpu_fused.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or attention or encq or cfg3 or encode or encoder" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; exit $rc; }
for r in 1 2 3; do
  for L in $P $X; do
    echo "== $(basename $L)" >> $O/ab.log
    QTX_LIB_PATH=$L timeout -k 10 100 python tools/attn_bench.py >> $O/ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/ab.log
for L in $P $X; do
  QTX_LIB_PATH=$L timeout -k 10 200 python tools/enc_bench.py 2>&1 | grep -i encoder | sed "s|^|$(basename $L) |" || exit 1
done
