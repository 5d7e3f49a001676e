#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel trace + PMC passes of the bench
# command (roofline kernel), the bench variants (serving cache, concurrency 1), phase traces.
# Set SKIP_TESTS=1 to skip pytest, AGG=1 to also profile the config-5 aggregation benchmark.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
fi
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
timeout -k 10 200 python bench.py --serving-cache --no-scale --no-cpu-baseline > gpurun_out/bench_serving.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_serving.log; exit 1; }
timeout -k 10 200 python bench.py --concurrent 1 --no-scale --no-cpu-baseline > gpurun_out/bench_c1.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_c1.log; exit 1; }
timeout -k 10 120 python tools/phasetrace.py icews14s_lgcn_roth "" 0 > gpurun_out/trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/trace.log; exit 1; }
# the profiled command runs one predict at a time, so the per-kernel durations match the
# live (isolated) HIP-event averages of the bench line
B="python bench.py --no-cpu-baseline --no-scale --concurrent 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- $B > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- $B --steps 48 > gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- $B --steps 48 > gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
if [ -n "$AGG" ]; then
timeout -k 10 600 python tools/aggbench.py --cpu --json gpurun_out/aggbench.json > gpurun_out/aggbench.log 2>&1 || { echo "aggbench failed"; exit 1; }
A="python tools/aggbench.py --reps 2"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/agg_prof -o run -- $A > gpurun_out/agg_prof.log 2>&1 || { echo "agg rocprof failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/agg_fetch -o run -- $A > gpurun_out/agg_fetch.log 2>&1 || { echo "agg pmc fetch failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/agg_write -o run -- $A > gpurun_out/agg_write.log 2>&1 || { echo "agg pmc write failed"; exit 1; }
fi
echo "all ok"
