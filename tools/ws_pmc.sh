#!/bin/bash
# PMC passes over the weight-stationary GEMM (one launch kind): tools/ws_pmc.sh <tag> <which>
set -o pipefail
T=${1:-wspmc}; W=${2:-qkv}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_IFETCH"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace -d $O/p$i -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/ws_one.py $W 5 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; }
done
echo done
