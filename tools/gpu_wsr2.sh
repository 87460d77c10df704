#!/bin/bash
# One GPU call: the O-projection at the decode's encoder M (cfg2: B=32, S=72 -> M=2304 and
# cfg5: M=18432): k_gemm_ws<RE_RES_LN> (default) vs k_gemm_wsr (QTX_WSR=1), encoder time
# and the cfg2 decode.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-wsr2}
mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in 0 1 0 1; do
  QTX_WSR=$v timeout -k 10 120 python tools/enc_small.py >> $O/enc_$v.log 2>&1 || { tail $O/enc_$v.log; exit 1; }
done
grep -H encoder $O/enc_*.log
for v in 0 1; do
  QTX_WSR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-cfg3 --steps 10 > $O/b_$v.json 2>$O/b_$v.err || { tail $O/b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$v.json')); print('QTX_WSR=$v', d['ms_per_step'])"
done
