#!/bin/bash
# round 4: the short row-scale chain in k_gemm_wsq (scale127 / rcp_cr, no bpermute):
# the exhaustive exactness probe of the two forms, the GPU tests on the product library,
# then the encoder GEMM A/B against libqtx_x3.so (the previous HEAD), alternated
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-sc_ab}; mkdir -p $O
timeout -k 10 120 ./tools/probe_scale_exact > $O/scale_exact.log 2>&1; rc=$?
cat $O/scale_exact.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_status.py tests/test_gpu_configs.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 500 python tools/lib_ab.py onnx-transformer_amd/qtx/libqtx.so onnx-transformer_amd/qtx/libqtx_x3.so --rounds 4 > $O/lib_ab.log 2>&1; rc=$?
grep -v amdgpu.ids $O/lib_ab.log; exit $rc
