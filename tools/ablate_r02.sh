#!/bin/bash
# In-graph marginal cost of each decode kernel class (QTX_ABLATE bits, see csrc/qtx_api.hip):
# nop=1 replaces the class by an empty kernel (body cost), nop=0 drops it (body + boundary).
O=${1:-gpurun_out/abl}
mkdir -p $O
for nop in 1 0; do
  for bits in 0 2 4 8 16 32 128 256; do
    QTX_ABLATE=$bits QTX_ABLATE_NOP=$nop timeout -k 10 120 python bench.py --steps 4 --warmup 2 \
      --no-cpu-baseline --no-cfg3 > $O/abl_${nop}_${bits}.json 2> $O/abl_err.log || { echo "fail $nop $bits"; tail $O/abl_err.log; exit 1; }
    python -c "import json; d=json.loads(open('$O/abl_${nop}_${bits}.json').read().strip().splitlines()[-1]); print('nop=$nop ablate=$bits', round(d['ms_per_step']/71*1000,2), 'us/step')"
  done
done
