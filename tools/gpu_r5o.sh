#!/bin/bash
# round 5: owner-partition simulation over pipeline chunks per rank x chunk-tail streams
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "4 4" "8 4" "8 3"; do
  set -- $cfg
  REGCN_CHUNK_TAIL_STREAMS=$2 timeout -k 10 300 python -u tools/simprobe.py --world 8 --chunks $1 > gpurun_out/r5o_c$1_s$2.json 2> gpurun_out/r5o_c$1_s$2.err || { echo "sim $cfg failed"; tail -20 gpurun_out/r5o_c$1_s$2.err; exit 1; }
  python3 -c "
import json;o=json.load(open('gpurun_out/r5o_c$1_s$2.json'))
print('chunks $1 streams $2', {k:o[k] for k in ('max_rank_ms','replicated_ms','exposed_exchange_ms_per_step','predicted_step_ms')})" | tee -a gpurun_out/r5o.txt
done
echo "all ok"
