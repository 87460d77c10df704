#!/bin/bash
# One GPU call: tools/ws_diag.py for QTX_WSQ=2 and =1.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-wsdiag}
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/ws_diag.py 2 300 4096 > $O/diag2.log 2>&1; rc=$?
cat $O/diag2.log | head -80
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ws_diag.py 1 300 > $O/diag1.log 2>&1; rc=$?
cat $O/diag1.log; exit $rc
