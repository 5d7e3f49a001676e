set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 48 --warmup 4 > gpurun_out/b2.log 2>&1 || { echo "2-rank failed"; tail -30 gpurun_out/b2.log; exit 1; }
grep '^{' gpurun_out/b2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["n_gpus"], d["ms_per_step"], d["config"]["parallelism"])'
