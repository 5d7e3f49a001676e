#!/bin/bash
# round 5: the default bench line (N=1) and the kernel trace of the same default command
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u bench.py > gpurun_out/r5i_bench.json 2> gpurun_out/r5i_bench.err || { echo "bench failed"; tail -20 gpurun_out/r5i_bench.err; exit 1; }
tail -c 600 gpurun_out/r5i_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5i_prof -o run -- python3 bench.py --no-extras --no-scale --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/r5i_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/r5i_prof.log; exit 1; }
echo "all ok"
