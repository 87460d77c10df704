set -o pipefail
mkdir -p gpurun_out/grp
for g in 1 2 4; do
  for gs in 71; do
    QTX_DECODE_GROUPS=$g timeout -k 10 200 python bench.py --no-cpu-baseline --no-cfg3 --steps 10 > gpurun_out/grp/g$g.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/grp/g$g.json')); print('groups $g', d['ms_per_step'], d['cfg5_per_gpu_decode'] if 'cfg5_per_gpu_decode' in d else '')"
  done
done
