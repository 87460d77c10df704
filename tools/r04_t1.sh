#!/bin/bash
# round 4: the f32-split probe, then the -m gpu suite + smoke on the product library
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04t1
timeout -k 10 60 ./tools/probe_f32_split > gpurun_out/r04t1/probe_f32_split.log 2>&1 || exit 1
cat gpurun_out/r04t1/probe_f32_split.log
bash tools/gpu_tests.sh r04t1
