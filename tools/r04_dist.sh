#!/bin/bash
# round 4: the driver's torchrun launch form at N=1 (RCCL backend) and the 2-rank flow
# rehearsed with gloo on the one GPU (sharding, max-over-ranks timing, id gather)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dist}; mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $O/torchrun1.json 2> $O/torchrun1.err || { tail $O/torchrun1.err; exit 1; }
tail -1 $O/torchrun1.json | head -c 400; echo
QTX_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --global-batch 512 --no-cpu-baseline --no-cfg3 > $O/gloo2.json 2> $O/gloo2.err || { tail $O/gloo2.err; exit 1; }
tail -1 $O/gloo2.json | head -c 400; echo
