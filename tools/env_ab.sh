#!/bin/bash
# A/B of HIP runtime environment knobs on the cfg2 decode (bench.py, decode line only).
set -o pipefail
mkdir -p gpurun_out/env
run() {
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-cfg3 --steps 10 > gpurun_out/env/b.json 2>/dev/null || return 1
  python -c "import json; d=json.load(open('gpurun_out/env/b.json')); print('$*', round(d['ms_per_step'], 3))"
}
run X=0 || exit 1
run HIP_FORCE_DEV_KERNARG=1 || exit 1
run HIP_FORCE_DEV_KERNARG=0 || exit 1
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
run X=0 || exit 1
