#!/bin/bash
# round 5: the owner simulation with the longer blocker and the collector off while enqueuing
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5x.json 2> gpurun_out/r5x.err || { echo "sim failed"; tail -20 gpurun_out/r5x.err; exit 1; }
python3 -c "
import json;o=json.load(open('gpurun_out/r5x.json'))
print({k:o[k] for k in ('per_rank_ms','max_rank_ms','replicated_ms','exposed_exchange_ms_per_step','predicted_step_ms','blocker_margin_ms')})"
echo "all ok"
