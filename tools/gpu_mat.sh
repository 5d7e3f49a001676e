#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rowtail.py tests/test_gpu_config5_pin.py tests/test_gpu_parity.py tests/test_gpu_scale.py > gpurun_out/pytest_mat.log 2>&1 || { echo "tests failed"; grep -E "Error|assert|FAILED" gpurun_out/pytest_mat.log | head; tail -3 gpurun_out/pytest_mat.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/pytest_mat.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mat_prof -o run -- python tools/c5probe.py --modes layers --reps 3 > gpurun_out/mat_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/mat_prof.log; exit 1; }
grep "ms per predict" gpurun_out/mat_prof.log
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/mat_prof/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('rowtail', 'gather_agg', 'union_runs', 'score')):
        print("   %-60s %5s %9.1f us" % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY
