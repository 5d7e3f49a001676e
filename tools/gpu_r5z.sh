#!/bin/bash
# round 5: the 8-rank simulation with the crel gather limited to views of >= 768 big tiles
# (REGCN_CREL_MIN_TILES; a rank's view has ~220) vs the default
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 768 0 768 0; do
  REGCN_CREL_MIN_TILES=$v timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5z_sim$v.json 2> gpurun_out/r5z_sim$v.err || { echo "sim $v failed"; tail -20 gpurun_out/r5z_sim$v.err; exit 1; }
  python3 -c "
import json;o=json.load(open('gpurun_out/r5z_sim$v.json'))
print('crel_min_tiles=$v', {k:o[k] for k in ('max_rank_ms','replicated_ms','exposed_exchange_ms_per_step','predicted_step_ms')})" | tee -a gpurun_out/r5z.txt
done
echo "all ok"
