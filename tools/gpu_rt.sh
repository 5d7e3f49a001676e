#!/bin/bash
# rowtail check: its parity tests, then per-predict times of config 5 (fused k_layer vs the
# rowtail, one stream vs chunk-pipelined) and kernel times of the pipelined rowtail.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_rowtail.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_rt.log 2>&1 || { echo "rowtail tests failed"; tail -30 gpurun_out/pytest_rt.log; exit 1; }
tail -1 gpurun_out/pytest_rt.log
for cfg in "fused 100000000 1" "rt1 65536 1" "rt4 65536 4" "rt8 65536 8"; do
  set -- $cfg
  REGCN_ROWTAIL_MIN_ROWS=$2 REGCN_ROWTAIL_CHUNKS=$3 timeout -k 10 200 python tools/c5probe.py --modes layers --reps 5 > gpurun_out/rt_$1.log 2>&1 || { echo "probe $1 failed"; tail -20 gpurun_out/rt_$1.log; exit 1; }
  echo "$1: $(grep 'ms per predict' gpurun_out/rt_$1.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rt_prof -o run -- python tools/c5probe.py --modes layers --reps 3 > gpurun_out/rt_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/rt_prof.log; exit 1; }
grep "ms per predict" gpurun_out/rt_prof.log
