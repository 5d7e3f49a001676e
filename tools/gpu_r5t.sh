#!/bin/bash
# round 5: the owner partition's per-rank initial state -- sharded GPU tests, then the
# 8-rank simulation with it off / on
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r5t_pytest.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5t_pytest.log; exit 1; }
tail -2 gpurun_out/r5t_pytest.log
for oi in 0 1 0 1; do
  REGCN_OWNER_INIT=$oi timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5t_oi$oi.json 2> gpurun_out/r5t_oi$oi.err || { echo "sim $oi failed"; tail -20 gpurun_out/r5t_oi$oi.err; exit 1; }
  python3 -c "
import json;o=json.load(open('gpurun_out/r5t_oi$oi.json'))
print('owner_init $oi', {k:o[k] for k in ('max_rank_ms','replicated_ms','exposed_exchange_ms_per_step','predicted_step_ms')})" | tee -a gpurun_out/r5t.txt
done
echo "all ok"
