#!/bin/bash
# round 4: weight-stationary candidate libqtx_x3.so — its bit-exact GPU tests, the encoder
# GEMM A/B against the product library (alternated), the stamped QKV / FFN1 phases
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ws_ab}; mkdir -p $O
X=onnx-transformer_amd/qtx/libqtx_x3.so
QTX_LIB_PATH=$X timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_status.py tests/test_gpu_configs.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_x.log 2>&1; rc=$?
tail -2 $O/pytest_x.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_x.log | head; exit $rc; }
timeout -k 10 600 python tools/lib_ab.py onnx-transformer_amd/qtx/libqtx.so $X --rounds 5 > $O/lib_ab.log 2>&1; rc=$?
grep -v amdgpu.ids $O/lib_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/wsq_stamps.py 1 2>&1 | grep -v amdgpu.ids | tee $O/qkv_stamps.log || exit 1
timeout -k 10 200 python tools/wsq_stamps.py ffn1 2>&1 | grep -v amdgpu.ids | tee $O/ffn1_stamps.log
