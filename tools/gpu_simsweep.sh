#!/bin/bash
# owner-partition rank simulation (8 ranks) under environment variants: VARS="A=1 B=2;C=3" (';' separates runs)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
IFS=';' read -ra RUNS <<< "${VARS:-}"
[ ${#RUNS[@]} -eq 0 ] && RUNS=("")
i=0
for v in "${RUNS[@]}"; do
  echo "== $v" | tee -a $R/gpurun_out/simsweep.log
  env $v timeout -k 10 300 python3 $R/tools/simprobe.py --world 8 ${SIMARGS:-} > $R/gpurun_out/simsweep_$i.json 2>> $R/gpurun_out/simsweep.log || exit 1
  python3 -c "import json;d=json.load(open('$R/gpurun_out/simsweep_$i.json'));print('$v', d['max_rank_ms'], d['mean_rank_ms'], d['replicated_ms'], d['predicted_step_ms'], [round(x,3) for x in d['per_rank_encoder_ms']][:2], d['per_rank_decoder_ms'][:2])" | tee -a $R/gpurun_out/simsweep.log
  i=$((i+1))
done
