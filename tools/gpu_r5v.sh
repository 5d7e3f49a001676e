#!/bin/bash
# round 5: sharded GPU tests, then the 8-rank owner simulation (twice) after the relation-means
# split (ranks' sums -> one stand-in all_reduce -> the division)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r5v_pytest.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5v_pytest.log; exit 1; }
tail -2 gpurun_out/r5v_pytest.log
for n in 1 2; do
  timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5v_$n.json 2> gpurun_out/r5v_$n.err || { echo "sim failed"; tail -20 gpurun_out/r5v_$n.err; exit 1; }
  python3 -c "
import json;o=json.load(open('gpurun_out/r5v_$n.json'))
print('run $n', {k:o[k] for k in ('max_rank_ms','replicated_ms','exposed_exchange_ms_per_step','predicted_step_ms')})" | tee -a gpurun_out/r5v.txt
done
echo "all ok"
