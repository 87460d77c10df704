#!/bin/bash
# One GPU call: the MFMA/VALU issue probe (tools/probe_mfma_valu.hip), then tools/gpu_round.sh.
set -o pipefail
T=${1:-run}
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/$T
timeout -k 10 120 $GRAFT_REPO_ROOT/tools/probe_mfma_valu > $GRAFT_REPO_ROOT/gpurun_out/$T/probe_mfma_valu.log 2>&1 || { echo probe failed; cat $GRAFT_REPO_ROOT/gpurun_out/$T/probe_mfma_valu.log; exit 1; }
cat $GRAFT_REPO_ROOT/gpurun_out/$T/probe_mfma_valu.log
bash $GRAFT_REPO_ROOT/tools/gpu_round.sh "$@"
