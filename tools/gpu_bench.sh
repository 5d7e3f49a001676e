#!/bin/bash
# headline bench (default N=1 run: config 5 + extras), then a rocprof kernel-stats pass of a short bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
tail -c 600 gpurun_out/bench.json; echo
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bench_prof -o run -- python -u bench.py --steps 6 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { echo "rocprof bench failed"; tail -10 gpurun_out/bench_prof.err; exit 1; }
tail -c 300 gpurun_out/bench_prof.json
