#!/bin/bash
# 2-rank rehearsal of the config-5 owner partition on one card (gloo), as the driver launches bench.py
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
BENCH_DIST_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps ${STEPS:-3} --warmup 1 ${ARGS:-} \
  > $R/gpurun_out/w2.json 2> $R/gpurun_out/w2.err
