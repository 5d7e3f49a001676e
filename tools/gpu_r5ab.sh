#!/bin/bash
# round 5: owner-partition simulation at 3 and 2 pipeline chunks per rank vs the default 4
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in 3 2 4 3; do
  timeout -k 10 300 python -u tools/simprobe.py --world 8 --chunks $c > gpurun_out/r5ab_c$c.json 2> gpurun_out/r5ab_c$c.err || { echo "sim $c failed"; tail -20 gpurun_out/r5ab_c$c.err; exit 1; }
  python3 -c "
import json;o=json.load(open('gpurun_out/r5ab_c$c.json'))
print('chunks $c', {k:o[k] for k in ('max_rank_ms','replicated_ms','exposed_exchange_ms_per_step','predicted_step_ms')})" | tee -a gpurun_out/r5ab.txt
done
echo "all ok"
