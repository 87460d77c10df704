#!/bin/bash
# round-4 first GPU call: the baseline round at HEAD, then the fast-epilogue A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh r04a || exit 1
mkdir -p gpurun_out/r04a
timeout -k 10 400 python tools/lib_ab.py onnx-transformer_amd/qtx/libqtx.so onnx-transformer_amd/qtx/libqtx_diag.so --rounds 2 > gpurun_out/r04a/lib_ab.log 2>&1; rc=$?
cat gpurun_out/r04a/lib_ab.log; exit $rc
