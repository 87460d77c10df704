#!/bin/bash
# A/B of the N-split skinny GEMM (QTX_SKINNY_WIDE=<rows per WG>): parity, per-kernel in-graph
# cost, decode time.
set -o pipefail
O=gpurun_out/wide; mkdir -p $O
QTX_SKINNY_WIDE=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_model.py tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest4.log 2>&1 || { tail -30 $O/pytest4.log; exit 1; }
tail -1 $O/pytest4.log
QTX_SKINNY_WIDE=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest8.log 2>&1 || { tail -30 $O/pytest8.log; exit 1; }
tail -1 $O/pytest8.log
for w in 0 4 8; do
  QTX_SKINNY_WIDE=$w timeout -k 10 120 python tools/kernel_chain.py 2>&1 | grep -v amdgpu.ids | sed "s/^/wide=$w /" || exit 1
  QTX_SKINNY_WIDE=$w timeout -k 10 200 python bench.py --no-cpu-baseline --no-cfg3 --steps 10 > $O/b$w.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/b$w.json')); print('wide=$w decode ms', round(d['ms_per_step'], 3))"
done
