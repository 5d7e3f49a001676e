#!/bin/bash
# Config-5 profiles: rocprofv3 kernel trace + PMC FETCH_SIZE / WRITE_SIZE of the headline bench
# command (WHICH=bench) or of the aggregation benchmark (WHICH=agg, UNIFORM=1 for uniform
# sources) or of the ICEWS14s bench command (WHICH=icews).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
case "$WHICH" in
  bench) T=c5; C="python bench.py --no-extras --no-scale --no-cpu-baseline --steps 6 --warmup 1";;
  agg) T=agg${UNIFORM:+_uniform}; C="python tools/aggbench.py --reps 2 --which union_aggregate,union_aggregate_src_runs,lorentz_aggregate ${UNIFORM:+--uniform-src}";;
  icews) T=ic; C="python bench.py --config icews14s_lgcn_roth --no-scale --no-cpu-baseline --concurrent 1 --steps 48";;
esac
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- $C > gpurun_out/${T}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o run -- $C > gpurun_out/${T}_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o run -- $C > gpurun_out/${T}_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
echo "profiles $T ok"
