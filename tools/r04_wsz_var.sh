#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-wszv}
mkdir -p $O
cd $GRAFT_REPO_ROOT
L=onnx-transformer_amd/qtx
QTX_WSQ=3 timeout -k 10 500 python tools/lib_ab.py $(ls $L/libqtx_s_*.so) --rounds 2 > $O/ab.log 2>&1; rc=$?
grep BEST $O/ab.log; exit $rc
