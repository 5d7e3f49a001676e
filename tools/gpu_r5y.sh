#!/bin/bash
# round 5: the crel gather beside the plain gather on a side stream (REGCN_CREL_SIDE=1 default vs 0):
# parity, headline A/B, the 8-rank simulation both ways
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_gpu_rowtail.py tests/test_gpu_sharded.py tests/test_gpu_scale.py -k "crel or rowtail or rank_simulation or world2 or scale" > gpurun_out/r5y_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r5y_pytest.log; exit 1; }
tail -1 gpurun_out/r5y_pytest.log
C="python -u bench.py --no-extras --no-scale --no-cpu-baseline --steps 10 --warmup 2"
for v in 1 0 1 0; do
  REGCN_CREL_SIDE=$v timeout -k 10 300 $C > gpurun_out/r5y_s$v.json 2> gpurun_out/r5y_s$v.err || { echo "bench $v failed"; tail -20 gpurun_out/r5y_s$v.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/r5y_s$v.json').read().strip().splitlines()[-1]);k=d['kernels']
print('side=$v', d['value'], d['ms_per_step'], 'gather %.1f' % k['regcn_layer_rowtail_f32(gather)']['avg_us'])" | tee -a gpurun_out/r5y.txt
done
for v in 1 0; do
  REGCN_CREL_SIDE=$v timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5y_sim$v.json 2> gpurun_out/r5y_sim$v.err || { echo "sim $v failed"; tail -20 gpurun_out/r5y_sim$v.err; exit 1; }
  python3 -c "
import json;o=json.load(open('gpurun_out/r5y_sim$v.json'))
print('sim side=$v', {k:o[k] for k in ('max_rank_ms','replicated_ms','exposed_exchange_ms_per_step','predicted_step_ms')})" | tee -a gpurun_out/r5y.txt
done
echo "all ok"
