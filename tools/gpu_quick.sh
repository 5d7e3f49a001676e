#!/bin/bash
# Quick GPU iteration: parity tests (optional), headline bench without the config-5 legs,
# concurrency-1 bench, no-memo phase trace.  TESTS=1 runs the GPU suite first.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$TESTS" ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
fi
for v in "" "--concurrent 1"; do
timeout -k 10 200 python bench.py $v --no-scale --no-cpu-baseline > gpurun_out/bq.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bq.log; exit 1; }
grep '^{' gpurun_out/bq.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$v"'", d["value"], d["ms_per_step"], d["latency_ms_per_predict"], " ".join("%s=%.2f" % (k, v["avg_us"]) for k, v in d["kernels"].items()))'
done
timeout -k 10 120 python tools/phasetrace.py icews14s_lgcn_roth "" 0 > gpurun_out/trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/trace.log; exit 1; }
cat gpurun_out/trace.log | grep -v amdgpu.ids
echo "all ok"
