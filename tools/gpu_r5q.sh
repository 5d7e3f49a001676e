#!/bin/bash
# round 5: 8-wave tiles with the deeper weight ring (phases; k_layer keeps 8 steps): parity,
# ICEWS14s bench, training sample, ICEWS14s kernel trace + FETCH / WRITE passes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_gpu_training.py -k "phase or layer or golden or shared_parameter or relation_gru or train" > gpurun_out/r5q_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r5q_pytest.log; exit 1; }
tail -1 gpurun_out/r5q_pytest.log
timeout -k 10 200 python -u bench.py --config icews14s_lgcn_roth --no-scale --no-cpu-baseline --steps 64 > gpurun_out/r5q_ic.json 2> gpurun_out/r5q_ic.err || { echo "ic bench failed"; tail -20 gpurun_out/r5q_ic.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r5q_ic.json').read().strip().splitlines()[-1])
print(d['value'], d['latency_ms_per_predict'], {k: v['avg_us'] for k, v in d['kernels'].items()}, d['breakdown']['encoder_kernels_us_per_step'])"
timeout -k 10 200 python -u tools/trainbench.py --graph --no-cpu > gpurun_out/r5q_train.log 2>&1 || { echo "trainbench failed"; tail -20 gpurun_out/r5q_train.log; exit 1; }
tail -3 gpurun_out/r5q_train.log
WHICH=icews bash tools/gpu_prof_c5.sh
echo "all ok"
