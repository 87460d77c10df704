#!/bin/bash
# decode-path check + timing in one GPU call: the decode / attention / config GPU tests,
# the stamped per-phase decode kernels, then the bench line (no CPU baseline, no cfg3).
# usage: tools/gpu_dec.sh <tag>
T=${1:-dec}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_model.py tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_fault.py tests/test_trace.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 150 python tools/stamp_bench.py > $O/stamps.log 2>&1 || { echo stamps failed; tail $O/stamps.log; exit 1; }
grep dec_attn $O/stamps.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-cfg3 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('tok/s', round(d['value']), 'ms', round(d['ms_per_step'], 3), 'step_us', round(d['step']['us'], 1))"
