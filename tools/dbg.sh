set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in 4 1; do
timeout -k 10 200 python -X faulthandler bench.py --concurrent $c --no-scale --no-cpu-baseline > gpurun_out/dbg$c.log 2>&1 || { echo "c$c failed"; tail -20 gpurun_out/dbg$c.log; exit 1; }
grep '^{' gpurun_out/dbg$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c='$c'", d["value"], d["ms_per_step"], d["latency_ms_per_predict"], " ".join("%s=%.2f" % (k, v["avg_us"]) for k, v in d["kernels"].items()))'
done
