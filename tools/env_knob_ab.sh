#!/bin/bash
# GPU parity tests, then an A/B of one environment knob on the in-graph kernel costs
# (tools/kernel_chain.py) and the cfg2 decode (bench.py):  tools/env_knob_ab.sh VAR VALUE_A VALUE_B
set -o pipefail
V=$1; A=$2; B=$3
mkdir -p gpurun_out/ab
[ -n "$NOTEST" ] || timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/ab/t.log 2>&1 || { tail -30 gpurun_out/ab/t.log; exit 1; }
tail -1 gpurun_out/ab/t.log
if [ -z "$NOCHAIN" ]; then for v in $A $B; do
  echo "$V=$v"; env $V=$v timeout -k 10 120 python tools/kernel_chain.py 2>&1 | grep -E "attn|FFN2|layer as" || exit 1
done; fi
run() {
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-cfg3 --steps 10 $BARGS > gpurun_out/ab/b.json 2>/dev/null || return 1
  python -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print('$*', round(d['ms_per_step'], 3), 'B', d['config']['per_gpu_batch'])"
}
for i in 1 2; do run $V=$A || exit 1; run $V=$B || exit 1; done
