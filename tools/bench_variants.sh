#!/bin/bash
# ms per decode of bench.py under several QTX_* experiment settings: "NAME=VAL,NAME=VAL ..."
for v in "$@"; do
  env $(echo "$v" | tr ',' ' ') timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
    --no-cpu-baseline --no-cfg3 > gpurun_out/bv.json 2> /dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/bv.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'], 3), 'ms', int(d['value']), 'tok/s')"
done
