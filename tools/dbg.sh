set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "--pool 16" "" "--pool 16" ""; do
timeout -k 10 200 python bench.py $v --no-scale --no-cpu-baseline > gpurun_out/dbg.log 2>&1 || { echo "$v failed"; tail -20 gpurun_out/dbg.log; exit 1; }
grep '^{' gpurun_out/dbg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$v"'", d["value"], d["ms_per_step"], d["latency_ms_per_predict"])'
done
