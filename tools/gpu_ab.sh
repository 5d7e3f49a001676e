#!/bin/bash
# A/B of environment variants on the config-5 headline (short runs): VARS="A=1;A=2" (';' separates runs)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R
IFS=';' read -ra RUNS <<< "${VARS:-}"
i=0
for v in "${RUNS[@]}"; do
  env $v timeout -k 10 400 python3 -u bench.py --steps ${STEPS:-8} --warmup 2 --no-extras --no-cpu-baseline ${ARGS:-} > $R/gpurun_out/ab_$i.json 2> $R/gpurun_out/ab_$i.err || exit 1
  python3 - "$v" $R/gpurun_out/ab_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
pick = {n: v["avg_us"] for n, v in k.items() if n in ("regcn_union_aggregate_src_runs_f32", "regcn_segment_mean_f32", "regcn_layer_rowtail_f32(gather)", "regcn_layer_rowtail_f32", "regcn_layer_rowtail_f32(step)", "regcn_hyp_score_jobs_f32")}
print(sys.argv[1], d["value"], d["ms_per_step"], pick, flush=True)
PY
  i=$((i+1))
done
