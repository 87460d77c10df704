#!/bin/bash
# weight-stationary variants (QTX_WSQ=3: k_gemm_wsz, 4: k_gemm_wsa; QTX_WSA2: FFN1 two-pass): tests, A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-wsz}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v --timeout 120 --timeout-method thread -k "ws_qkv_scales or splitk_bad or twopass_wsa2" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python tools/gemm_ab.py QTX_WSQ=1 QTX_WSQ=3 QTX_WSQ=4 QTX_WSQ=4,QTX_WSA2=1,QTX_BENCH_FFN1_2PASS=1 QTX_WSQ=1,QTX_BENCH_FFN1_2PASS=1 --reps 3 > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
cat $O/ab.log
