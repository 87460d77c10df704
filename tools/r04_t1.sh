#!/bin/bash
# round 4: the f32-split probe, then the -m gpu suite + smoke on the product library
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04t1
true && {
}
bash tools/gpu_tests.sh r04t1
