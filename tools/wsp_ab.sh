#!/bin/bash
# A/B of the pipelined weight-stationary GEMM variants (QTX_WSP): parity tests, then per
# variant the cfg3 launch times (bench.time_row_gemms) and the stamped phase breakdown.
# usage: tools/wsp_ab.sh <tag> [variants...]
set -o pipefail
T=${1:-wsp}; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "linear_rows_ws or pack_w_ws" -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in ${@:-default}; do
  QTX_WSP=$v timeout -k 10 120 python -c "
import bench
r = bench.time_row_gemms(reps=20)
print('$v', ' '.join(f'{k} {v[0]:.1f}' for k, v in r.items()), flush=True)" >> $O/times.log 2>&1 || { tail $O/times.log; exit 1; }
  QTX_WSP=$v timeout -k 10 120 python tools/wsp_stamps.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/stamps.log || exit 1
done
cat $O/times.log $O/stamps.log
