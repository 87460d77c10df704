#!/bin/bash
# One GPU call: the weight-stationary GEMM tests (all kernels), the QKV A/B timing and stamps.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-wsq}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v --timeout 120 --timeout-method thread -k "${2:-ws}" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python tools/gemm_ab.py ${3:-QTX_WSQ=0 QTX_WSQ=1 QTX_WSQ=2} --reps 3 > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 120 python tools/wsq_stamps.py ${4:-} > $O/stamps.log 2>&1; rc=$?
cat $O/stamps.log; exit $rc
