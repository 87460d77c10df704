#!/bin/bash
# One GPU call: the weight-stationary GEMM tests (all kernels) and the encoder GEMM A/B
# of the one-pass FFN1 kernels (QTX_WSY=0: k_gemm_wsx, 1: k_gemm_wsy).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-wsy}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v --timeout 120 --timeout-method thread -k "ws" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python tools/gemm_ab.py QTX_WSY=0 QTX_WSY=1 --reps 3 > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
cat $O/ab.log
