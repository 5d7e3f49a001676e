#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/graphdbg2.py > gpurun_out/graphdbg2.log 2>&1 || { echo "graphdbg2 failed"; tail -30 gpurun_out/graphdbg2.log; exit 1; }
tail -16 gpurun_out/graphdbg2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rt1_prof -o run -- python tools/c5probe.py --modes layers --reps 3 > gpurun_out/rt1_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/rt1_prof.log; exit 1; }
grep "ms per predict" gpurun_out/rt1_prof.log
