#!/bin/bash
# One GPU call: MFMA/VALU issue probe (mixed and specialised waves) + the 32x32 layout check.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-probe}
mkdir -p $O
timeout -k 10 120 $GRAFT_REPO_ROOT/tools/probe_mfma32_layout > $O/layout.log 2>&1; echo "layout rc=$?"; cat $O/layout.log
timeout -k 10 180 $GRAFT_REPO_ROOT/tools/probe_mfma_valu > $O/probe_mfma_valu.log 2>&1 || { echo probe failed; cat $O/probe_mfma_valu.log; exit 1; }
cat $O/probe_mfma_valu.log
