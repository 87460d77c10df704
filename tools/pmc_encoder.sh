#!/bin/bash
# rocprofv3 over the cfg3 encoder exactly as the product runs it (tools/enc_profile.py):
# kernel stats, then one PMC pass per counter group (never combined with tracing).
# usage: tools/pmc_encoder.sh <outdir under gpurun_out>
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc_enc}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python $GRAFT_REPO_ROOT/tools/enc_profile.py > $O/stats.log 2>&1 || { echo "stats failed"; tail -5 $O/stats.log; exit 1; }
i=0
for pmc in "MfmaUtil" "SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE" "LdsBankConflict"; do
  i=$((i + 1))
  echo "pass $i: $pmc"
  timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-trace -d $O/p$i -o run --output-format csv \
    -- python $GRAFT_REPO_ROOT/tools/enc_profile.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
echo done
