#!/bin/bash
# One GPU session, in two calls (each fits gpurun's limit):
#   PART=tests   the GPU suite and the default bench (config-5 headline + ICEWS legs)
#   PART=prof    rocprofv3 kernel traces and PMC (FETCH_SIZE / WRITE_SIZE) passes of the
#                config-5 bench command, the config-5 aggregation benchmark (Zipf and
#                uniform sources) and the ICEWS14s bench command
# Summaries: python tools/pmc_traffic.py <fetch dir> <write dir> --config ... > profiles/...
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$PART" = "tests" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
echo "tests + bench ok"
fi
if [ "$PART" = "prof" ]; then
B="python bench.py --no-extras --no-scale --no-cpu-baseline --steps 6 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5_prof -o run -- $B > gpurun_out/c5_prof.log 2>&1 || { echo "rocprof c5 failed"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c5_fetch -o run -- $B > gpurun_out/c5_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/c5_write -o run -- $B > gpurun_out/c5_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
A="python tools/aggbench.py --reps 2 --which union_aggregate,union_aggregate_src_runs,lorentz_aggregate"
for u in "" "--uniform-src"; do
  t=agg${u:+_uniform}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${t}_prof -o run -- $A $u > gpurun_out/${t}_prof.log 2>&1 || { echo "agg rocprof failed"; exit 1; }
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${t}_fetch -o run -- $A $u > gpurun_out/${t}_fetch.log 2>&1 || { echo "agg pmc fetch failed"; exit 1; }
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${t}_write -o run -- $A $u > gpurun_out/${t}_write.log 2>&1 || { echo "agg pmc write failed"; exit 1; }
done
S="python bench.py --config icews14s_lgcn_roth --no-scale --no-cpu-baseline --concurrent 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ic_prof -o run -- $S > gpurun_out/ic_prof.log 2>&1 || { echo "rocprof icews failed"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ic_fetch -o run -- $S --steps 48 > gpurun_out/ic_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ic_write -o run -- $S --steps 48 > gpurun_out/ic_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
echo "profiles ok"
fi
