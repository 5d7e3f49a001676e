set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "shared or phase" > gpurun_out/pt.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for v in "" "--concurrent 1" "" ; do
timeout -k 10 200 python bench.py $v --no-scale --no-cpu-baseline > gpurun_out/dbg.log 2>&1 || { echo "$v failed"; tail -20 gpurun_out/dbg.log; exit 1; }
grep '^{' gpurun_out/dbg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$v"'", d["value"], d["ms_per_step"], d["latency_ms_per_predict"], " ".join("%s=%.2f" % (k, v["avg_us"]) for k, v in d["kernels"].items()))'
done
