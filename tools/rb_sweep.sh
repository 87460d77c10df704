#!/bin/bash
# Decode row-block sweep (QTX_RB_* knobs of csrc/qtx_decode.hip skinny_mode): us per step.
for cfg in "4 4 8" "8 4 8" "4 8 8" "4 4 4" "4 4 16" "4 16 8"; do
  set -- $cfg
  QTX_RB_LN=$1 QTX_RB_F32Q=$2 QTX_RB_I8_512=$3 timeout -k 10 120 python bench.py --steps 4 --warmup 2 \
    --no-cpu-baseline --no-cfg3 > gpurun_out/rb.json 2> gpurun_out/rb.err || { echo "fail $cfg"; tail -3 gpurun_out/rb.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/rb.json').read().strip().splitlines()[-1]); print('RB_LN/F32Q/I8_512 = $cfg:', round(d['ms_per_step']/71*1000,2), 'us/step')"
done
