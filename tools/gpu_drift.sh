#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sharded.py -k rank_simulation > gpurun_out/pytest_sim.log 2>&1 || { echo "sim tests failed"; grep -E "Error|assert|FAILED" gpurun_out/pytest_sim.log | head; tail -3 gpurun_out/pytest_sim.log; exit 1; }
echo "sim tests: $(tail -1 gpurun_out/pytest_sim.log)"
timeout -k 10 300 python -u tools/graphdbg3.py > gpurun_out/graphdbg3.log 2>&1 || { echo "graphdbg3 failed"; tail -30 gpurun_out/graphdbg3.log; exit 1; }
grep -E "^key .*recorded|^graphs" gpurun_out/graphdbg3.log | cut -c1-1500
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_cli.py -k "hip_graph" > gpurun_out/pytest_drift.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|assert" gpurun_out/pytest_drift.log | head -20
[ $rc -eq 0 ] || exit $rc
for c in 1 2 4; do
  timeout -k 10 300 python tools/simprobe.py --world 8 --chunks $c > gpurun_out/sim_c$c.log 2>&1 || { echo "simprobe $c failed"; tail -20 gpurun_out/sim_c$c.log; exit 1; }
  echo "chunks=$c $(grep '^{' gpurun_out/sim_c$c.log | cut -c1-420)"
done
