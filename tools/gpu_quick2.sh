#!/bin/bash
# Round-4 check: the GPU suite, then a config-5 bench with the extras (ICEWS legs, owner simulation).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python -u bench.py --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:---no-cpu-baseline --no-scale} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -c 3000 gpurun_out/bench.log
