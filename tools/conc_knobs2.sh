#!/bin/bash
# One GPU call: sub-batch concurrency variants at B = 32 / 256 / 512 (ids checksums must
# agree per B): one graph (g1), G graphs on G streams (g2), one graph with G independent
# branches (joint: QTX_GROUP_GRAPH=1), eager launches on G streams (eager).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-knobs2}
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {  # name, batch, then env assignments
  local n=$1 b=$2; shift 2
  env "$@" timeout -k 10 200 python tools/decode_conc.py --batch $b --reps 5 > $O/$n.log 2>&1 || { tail $O/$n.log; return 1; }
  echo "$n: $(grep -h 'ms per decode' $O/$n.log)"
}
for B in 32 256 512; do
  run b${B}_g1 $B QTX_DECODE_GROUPS=1 &&
  run b${B}_g2 $B QTX_DECODE_GROUPS=2 &&
  run b${B}_joint2 $B QTX_DECODE_GROUPS=2 QTX_GROUP_GRAPH=1 &&
  run b${B}_joint4 $B QTX_DECODE_GROUPS=4 QTX_GROUP_GRAPH=1 &&
  run b${B}_eager2 $B QTX_DECODE_GROUPS=2 QTX_NO_GRAPH=1 || exit 1
done
