#!/bin/bash
# the whole GPU suite in one process, then smoke()
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_all.log
grep -E "FAILED|Error" gpurun_out/pytest_gpu_all.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?
tail -2 gpurun_out/smoke.log
exit $rc
