#!/bin/bash
# rocprofv3 PMC passes over the cfg3 QuantLinear launches (tools/rows_bench.py), one pass
# per counter group (never combined with tracing; MI355X_MICROARCH.md PMC slot limits).
# usage: tools/pmc_gemm.sh <outdir under gpurun_out>
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc_gemm}
mkdir -p $O
cd /tmp
i=0
for pmc in "MfmaUtil" "SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "FETCH_SIZE" "WRITE_SIZE" \
           "LdsBankConflict" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum"; do
  i=$((i + 1))
  echo "pass $i: $pmc"
  timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-trace -d $O/p$i -o run --output-format csv \
    -- python $GRAFT_REPO_ROOT/tools/rows_bench.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
echo done
