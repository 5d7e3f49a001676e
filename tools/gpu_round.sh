#!/bin/bash
# One GPU session: parity tests, microbench, bench, rocprof kernel trace + PMC passes of the
# bench command (roofline kernel) and of the config-5 aggregation benchmark.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python tools/microbench.py > gpurun_out/micro.log 2>&1 || { echo "micro failed"; tail -5 gpurun_out/micro.log; exit 1; }
timeout -k 10 120 python tools/microbench.py --trace > gpurun_out/trace.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/trace.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench.log; exit 1; }
B="python bench.py --no-cpu-baseline --no-scale"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- $B > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- $B --steps 50 > gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- $B --steps 50 > gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
timeout -k 10 600 python tools/aggbench.py --cpu --json gpurun_out/aggbench.json > gpurun_out/aggbench.log 2>&1 || { echo "aggbench failed"; exit 1; }
A="python tools/aggbench.py --reps 2"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/agg_prof -o run -- $A > gpurun_out/agg_prof.log 2>&1 || { echo "agg rocprof failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/agg_fetch -o run -- $A > gpurun_out/agg_fetch.log 2>&1 || { echo "agg pmc fetch failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/agg_write -o run -- $A > gpurun_out/agg_write.log 2>&1 || { echo "agg pmc write failed"; exit 1; }
echo "all ok"
