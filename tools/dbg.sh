set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "--concurrent 8 --pool 16" "--concurrent 6 --pool 12" "--serving-cache" "--serving-cache --concurrent 8 --pool 16"; do
timeout -k 10 200 python -X faulthandler bench.py $v --no-scale --no-cpu-baseline > gpurun_out/dbg.log 2>&1 || { echo "$v failed"; tail -20 gpurun_out/dbg.log; exit 1; }
grep '^{' gpurun_out/dbg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$v"'", d["value"], d["ms_per_step"], d["latency_ms_per_predict"], " ".join("%s=%.2f" % (k, v["avg_us"]) for k, v in d["kernels"].items()))'
done
