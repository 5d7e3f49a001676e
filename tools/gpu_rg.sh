#!/bin/bash
# rowtail row-group variants: parity (both), then config-5 per-predict time and kernel times
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rg in 1 2; do
  REGCN_ROWTAIL_RG=$rg timeout -k 10 300 python -u -m pytest tests/test_gpu_rowtail.py -q -x --timeout 250 --timeout-method thread > gpurun_out/pytest_rg$rg.log 2>&1 || { echo "rowtail tests rg=$rg failed"; grep -E "Error|assert|FAILED" gpurun_out/pytest_rg$rg.log | head; tail -3 gpurun_out/pytest_rg$rg.log; exit 1; }
  echo "rg=$rg $(tail -1 gpurun_out/pytest_rg$rg.log)"
done
for rg in 1 2; do
  REGCN_ROWTAIL_RG=$rg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rg${rg}_prof -o run -- python tools/c5probe.py --modes layers --reps 3 > gpurun_out/rg${rg}_prof.log 2>&1 || { echo "rocprof rg=$rg failed"; tail -20 gpurun_out/rg${rg}_prof.log; exit 1; }
  echo "rg=$rg $(grep 'ms per predict' gpurun_out/rg${rg}_prof.log)"
  python - $rg <<'PY'
import csv, sys
for r in csv.DictReader(open('gpurun_out/rg%s_prof/run_kernel_stats.csv' % sys.argv[1])):
    if any(k in r['Name'] for k in ('rowtail', 'gather_agg')):
        print("   %-60s %5s %9.1f us" % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "score or decoder or model" > gpurun_out/pytest_stagger.log 2>&1 || { echo "scorer tests failed"; grep -E "Error|assert|FAILED" gpurun_out/pytest_stagger.log | head; exit 1; }
echo "stagger tests: $(tail -1 gpurun_out/pytest_stagger.log)"
for sg in 0 1; do
  REGCN_SCORE_STAGGER=$sg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sg${sg}_prof -o run -- python tools/c5probe.py --modes layers --reps 3 > gpurun_out/sg${sg}_prof.log 2>&1 || { echo "rocprof sg=$sg failed"; tail -20 gpurun_out/sg${sg}_prof.log; exit 1; }
  python - $sg <<'PY'
import csv, sys
for r in csv.DictReader(open('gpurun_out/sg%s_prof/run_kernel_stats.csv' % sys.argv[1])):
    if 'score' in r['Name']:
        print("   stagger=%s %-50s %5s %9.1f us" % (sys.argv[1], r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
