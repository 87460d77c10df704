#!/bin/bash
# Per-launch in-graph cost of the decode kernels with the 8-wave FFN2 on and off.
set -o pipefail
mkdir -p gpurun_out/sk8
for v in 1 0 1 0; do
  echo "QTX_SKINNY8=$v"
  QTX_SKINNY8=$v timeout -k 10 120 python tools/kernel_chain.py 2>&1 | grep -E "FFN2|layer as" || exit 1
done
