#!/bin/bash
# One GPU call: kernel traces of (a) one process, B = 256, QTX_DECODE_GROUPS=2 (two sub-batch
# graphs on two streams), (b) the same with one group, (c) two processes at once, B = 256
# each; then tools/conc_analyze.py on each.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-conc}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
export QTX_DECODE_GROUPS=2
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/g2 -o run -- python $R/tools/decode_conc.py --batch 256 > $O/g2.log 2>&1 || { tail $O/g2.log; exit 1; }
export QTX_DECODE_GROUPS=1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/g1 -o run -- python $R/tools/decode_conc.py --batch 256 > $O/g1.log 2>&1 || { tail $O/g1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p0 -o run -- python $R/tools/decode_conc.py --batch 256 --reps 10 > $O/p0.log 2>&1 &
P0=$!
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p1 -o run -- python $R/tools/decode_conc.py --batch 256 --reps 10 --seed 1001 > $O/p1.log 2>&1 &
P1=$!
wait $P0; r0=$?
wait $P1; r1=$?
[ $r0 -eq 0 ] && [ $r1 -eq 0 ] || { tail $O/p0.log $O/p1.log; exit 1; }
# and untraced, for the wall times
timeout -k 10 300 python $R/tools/decode_conc.py --batch 256 --reps 10 > $O/u0.log 2>&1 &
P0=$!
timeout -k 10 300 python $R/tools/decode_conc.py --batch 256 --reps 10 --seed 1001 > $O/u1.log 2>&1 &
P1=$!
wait $P0; r0=$?
wait $P1; r1=$?
[ $r0 -eq 0 ] && [ $r1 -eq 0 ] || { tail $O/u0.log $O/u1.log; exit 1; }
grep -h "ms per decode" $O/*.log
cd $R
python tools/conc_analyze.py $O/g2 > $O/analysis.txt && python tools/conc_analyze.py $O/g1 >> $O/analysis.txt && python tools/conc_analyze.py $O/p0 $O/p1 >> $O/analysis.txt
cat $O/analysis.txt
