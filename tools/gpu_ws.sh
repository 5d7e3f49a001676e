#!/bin/bash
# wave-specialised scorer: parity tests, then kernel times of config-5 predicts with and without it
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_training.py > gpurun_out/pytest_ws.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_ws.log | head -30; tail -5 gpurun_out/pytest_ws.log; exit 1; }
tail -1 gpurun_out/pytest_ws.log
for ws in 0 1; do
  REGCN_SCORE_WS=$ws timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ws${ws}_prof -o run -- python tools/c5probe.py --modes layers --reps 3 > gpurun_out/ws${ws}_prof.log 2>&1 || { echo "rocprof $ws failed"; tail -20 gpurun_out/ws${ws}_prof.log; exit 1; }
  echo "ws=$ws $(grep 'ms per predict' gpurun_out/ws${ws}_prof.log)"
done
timeout -k 10 300 python -u tools/graphdbg2.py > gpurun_out/graphdbg2.log 2>&1 || { echo "graphdbg2 failed"; tail -30 gpurun_out/graphdbg2.log; exit 1; }
tail -16 gpurun_out/graphdbg2.log
