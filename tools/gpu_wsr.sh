#!/bin/bash
# One GPU call: weight-stationary GEMM tests and the encoder GEMM A/B: the O-projection
# (QTX_WS_RES_MAX_M=8192: KP row GEMM at cfg3's M; 1e9: k_gemm_wsr) and s_setprio 1 for
# waves 4-7 of k_gemm_wsq / k_gemm_wsy (QTX_WS_PRIO=1).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-wsr}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v --timeout 120 --timeout-method thread -k "ws" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python tools/gemm_ab.py QTX_WS_RES_MAX_M=8192 QTX_WS_RES_MAX_M=1000000000 QTX_WS_PRIO=1 --reps 3 > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
cat $O/ab.log
