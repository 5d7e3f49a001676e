#!/bin/bash
# round 5: step-tail staging at a constant row stride (no runtime division) A/B against the
# previous rowtail.hip (libregcn_hip_oldrt.so), plus the rowtail parity tests
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_rowtail.py tests/test_gpu_sharded.py -k "rowtail or rank_simulation" > gpurun_out/r5s_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r5s_pytest.log; exit 1; }
tail -1 gpurun_out/r5s_pytest.log
OLD=$GRAFT_REPO_ROOT/re-gcn_amd/regcn_amd/libregcn_hip_oldrt.so
C="python -u bench.py --no-extras --no-scale --no-cpu-baseline --steps 10 --warmup 2"
for v in new old new old; do
  if [ $v = old ]; then export REGCN_HIP_LIB=$OLD; else unset REGCN_HIP_LIB; fi
  timeout -k 10 300 $C > gpurun_out/r5s_$v.json 2> gpurun_out/r5s_$v.err || { echo "bench $v failed"; tail -20 gpurun_out/r5s_$v.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/r5s_$v.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$v', d['value'], d['ms_per_step'], 'rt2 %.1f rt3 %.1f' % (k['regcn_layer_rowtail_f32']['avg_us'], k['regcn_layer_rowtail_f32(step)']['avg_us']))" | tee -a gpurun_out/r5s.txt
done
echo "all ok"
