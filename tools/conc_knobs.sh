#!/bin/bash
# One GPU call: why two in-process sub-batch chains (QTX_DECODE_GROUPS=2) do not overlap —
# B = 256 decodes under runtime knobs, then a kernel trace of the most promising one.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-knobs}
mkdir -p $O
cd $GRAFT_REPO_ROOT
run() {  # name, then env assignments
  local n=$1; shift
  env "$@" timeout -k 10 200 python tools/decode_conc.py --batch 256 --reps 5 > $O/$n.log 2>&1 || { tail $O/$n.log; return 1; }
  echo "$n: $(grep -h 'ms per decode' $O/$n.log)"
}
run g1 QTX_DECODE_GROUPS=1 &&
run g2 QTX_DECODE_GROUPS=2 &&
run g2_nocap QTX_DECODE_GROUPS=2 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 &&
run g2_steps1 QTX_DECODE_GROUPS=2 QTX_GRAPH_STEPS=1 &&
run g2_q8 QTX_DECODE_GROUPS=2 GPU_MAX_HW_QUEUES=8 &&
run g2_eager QTX_DECODE_GROUPS=2 QTX_NO_GRAPH=1 &&
run g1_eager QTX_DECODE_GROUPS=1 QTX_NO_GRAPH=1 &&
run g2_eager_q8 QTX_DECODE_GROUPS=2 QTX_NO_GRAPH=1 GPU_MAX_HW_QUEUES=8 || exit 1
export TMPDIR=/tmp
cd /tmp
export QTX_DECODE_GROUPS=2 QTX_NO_GRAPH=1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/g2e -o run -- python $GRAFT_REPO_ROOT/tools/decode_conc.py --batch 256 --reps 3 > $O/g2e_trace.log 2>&1 || { tail $O/g2e_trace.log; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/conc_analyze.py $O/g2e | tee $O/analysis.txt
