#!/bin/bash
# One GPU call: the whole -m gpu suite, the bench line, rocprofv3 kernel stats of the
# bench, the dominant-kernel timing probe under rocprofv3, and the two PMC passes
# (FETCH_SIZE / WRITE_SIZE) over the dominant decode kernel.
# usage: tools/gpu_round.sh <tag> [pytest args...]   (outputs under gpurun_out/<tag>/)
set -o pipefail
T=${1:-run}; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
python -c "import sys; sys.path.insert(0, 'tools'); from prof_summary import sources_sha16; print(sources_sha16())" > $O/sources_sha16.txt
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAIL|Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tprobe -o run -- python $GRAFT_REPO_ROOT/tools/dominant_timing_probe.py > $O/tprobe.log 2>&1 || { echo tprobe failed; tail -20 $O/tprobe.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/pmc_dominant.py > $O/pmc1.log 2>&1 || { echo pmc1 failed; tail $O/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/pmc_dominant.py > $O/pmc2.log 2>&1 || { echo pmc2 failed; tail $O/pmc2.log; exit 1; }
echo done
