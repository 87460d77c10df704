#!/bin/bash
# One GPU call: parity tests, bench line, rocprofv3 kernel stats of the bench.
# usage: tools/gpu_check.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
T=${1:-run}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAIL|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo prof failed; tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo done
