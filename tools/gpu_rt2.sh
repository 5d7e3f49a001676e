#!/bin/bash
# rowtail parity + config-5 kernel times, then the graph-replay diagnostics
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_rowtail.py -q -x --timeout 250 --timeout-method thread > gpurun_out/pytest_rt.log 2>&1 || { echo "rowtail tests failed"; grep -E "Error|assert|FAILED" gpurun_out/pytest_rt.log | head; tail -3 gpurun_out/pytest_rt.log; exit 1; }
tail -1 gpurun_out/pytest_rt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rt2_prof -o run -- python tools/c5probe.py --modes layers --reps 3 > gpurun_out/rt2_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/rt2_prof.log; exit 1; }
grep "ms per predict" gpurun_out/rt2_prof.log
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/rt2_prof/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('rowtail', 'gather_agg', 'union_runs', 'score')):
        print("%-60s %5s %9.1f us" % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY
timeout -k 10 300 python -u tools/graphdbg3.py > gpurun_out/graphdbg3.log 2>&1 || { echo "graphdbg3 failed"; tail -30 gpurun_out/graphdbg3.log; exit 1; }
grep -E "^key .*recorded|^graphs" gpurun_out/graphdbg3.log | cut -c1-1500
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sim_prof -o run -- python tools/simprobe.py --world 8 > gpurun_out/sim_prof.log 2>&1 || { echo "simprobe failed"; tail -20 gpurun_out/sim_prof.log; exit 1; }
tail -1 gpurun_out/sim_prof.log | cut -c1-1500
