#!/bin/bash
# Round-end check as the driver runs it: GPU suite, smoke, default bench at --steps 20 and 200
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 500 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench20.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench20.log; exit 1; }
timeout -k 10 500 python -u bench.py --steps 200 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/bench200.log 2>&1 || { echo "bench200 failed"; tail -20 gpurun_out/bench200.log; exit 1; }
for f in bench20 bench200; do python -c "import json; j=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); print('$f', j['value'], j['ms_per_step'])"; done
