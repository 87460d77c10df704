#!/bin/bash
# In-graph cost of each kernel class of the fused decode step (see QTX_ABLATE in
# csrc/qtx_api.hip): drop the class (or replace it by an empty kernel) and time the bench.
export QTX_DECODE_GROUPS=${QTX_DECODE_GROUPS:-1}
for nop in ${NOPS:-1}; do
  for bits in 0 1 2 4 8 16 32 64 128 256 511; do
    QTX_ABLATE=$bits QTX_ABLATE_NOP=$nop timeout -k 10 120 python bench.py --steps 2 --warmup 1 \
      --no-cpu-baseline --no-cfg3 > gpurun_out/abl.json 2> /dev/null || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/abl.json').read().strip().splitlines()[-1]); print('nop=$nop ablate=$bits', round(d['ms_per_step']/71*1000,1), 'us/step')"
  done
done
