O=$GRAFT_REPO_ROOT/gpurun_out/r05h; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
i=0
for pmc in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-trace -d $O/p$i -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/ffn_one.py fused > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
echo done
