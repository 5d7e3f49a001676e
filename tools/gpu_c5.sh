#!/bin/bash
# Config-5 GPU session: parity tests of the aggregation / layer / model paths, the headline
# bench without the slow legs, the config-5 aggregation benchmark (Zipf and uniform sources,
# both edge orders).  K=<pytest -k expression> runs those GPU tests first.  FULL=1 adds the default bench (all legs).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$K" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
fi
timeout -k 10 300 python -u bench.py --no-extras --no-scale --no-cpu-baseline > gpurun_out/b5q.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b5q.log; exit 1; }
timeout -k 10 300 python -u tools/aggbench.py --which union_aggregate,union_aggregate_src_runs,union_layer --json gpurun_out/agg_zipf.json > gpurun_out/agg_zipf.log 2>&1 || { echo "aggbench failed"; tail -20 gpurun_out/agg_zipf.log; exit 1; }
timeout -k 10 300 python -u tools/aggbench.py --uniform-src --which union_aggregate,union_aggregate_src_runs,union_layer --json gpurun_out/agg_unif.json > gpurun_out/agg_unif.log 2>&1 || { echo "aggbench failed"; tail -20 gpurun_out/agg_unif.log; exit 1; }
if [ -n "$FULL" ]; then
timeout -k 10 600 python -u bench.py > gpurun_out/b5.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b5.log; exit 1; }
fi
echo "all ok"
