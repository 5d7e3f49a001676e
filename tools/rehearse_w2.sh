#!/bin/bash
# two ranks on the one card (gloo): the N > 1 bench paths end to end -- config 5 replicas with the
# owner-partition leg, then a dataset config (replicas + the edge-partition leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT/gpurun_out
export BENCH_DIST_BACKEND=gloo
BENCH_DETAIL=$R/w2_c5_detail.json timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 --no-extras --owner-leg \
  > $R/w2_c5.json 2> $R/w2_c5.err || { echo "w2 config 5 failed"; tail -20 $R/w2_c5.err; exit 1; }
tail -c 1500 $R/w2_c5.json
BENCH_DETAIL=$R/w2_gdelt_detail.json timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --config gdelt --steps 32 --warmup 1 --no-scale \
  > $R/w2_gdelt.json 2> $R/w2_gdelt.err || { echo "w2 gdelt failed"; tail -20 $R/w2_gdelt.err; exit 1; }
tail -c 800 $R/w2_gdelt.json
