#!/bin/bash
# round 5: phase B / C weight rings prefetched under the gather: bitwise phase tests, ICEWS14s bench, stage trace
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "phase or golden" > gpurun_out/r5r_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r5r_pytest.log; exit 1; }
tail -1 gpurun_out/r5r_pytest.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --config icews14s_lgcn_roth --no-scale --no-cpu-baseline --steps 64 > gpurun_out/r5r_ic$i.json 2> gpurun_out/r5r_ic$i.err || { echo "ic bench failed"; tail -20 gpurun_out/r5r_ic$i.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r5r_ic$i.json').read().strip().splitlines()[-1])
print(d['value'], d['latency_ms_per_predict'], {k: v['avg_us'] for k, v in d['kernels'].items()}, d['breakdown']['encoder_kernels_us_per_step'])"
done
timeout -k 10 200 python -u tools/phasetrace.py > gpurun_out/r5r_phasetrace.log 2>&1 || { echo "phasetrace failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/r5r_phasetrace.log | head -4
echo "all ok"
