#!/bin/bash
# the ring probe (tools/probe_ffn_ring.hip: the round-5 ring —
# every wave DMAs, one s_barrier per slot — against dedicated loader waves with FULL / FREE
# LDS words) timed, then rocprofv3 PMC passes over it (one counter group per run, no tracing
# besides --kernel-trace).  usage: tools/ring_probe.sh <outdir under gpurun_out>
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-ring}
mkdir -p $O
cd $GRAFT_REPO_ROOT/tools
[ -x probe_ffn_ring ] || hipcc --offload-arch=gfx950 -O3 -o probe_ffn_ring probe_ffn_ring.hip || exit 1
timeout -k 10 120 ./probe_ffn_ring > $O/probe.log 2>&1 || { echo "probe failed rc=$?"; tail -5 $O/probe.log; exit 1; }
cat $O/probe.log
cd /tmp
export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_I8" "LdsBankConflict"; do
  i=$((i + 1))
  echo "pass $i: $pmc"
  timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-trace -d $O/p$i -o run --output-format csv \
    -- $GRAFT_REPO_ROOT/tools/probe_ffn_ring pmc > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
echo done
