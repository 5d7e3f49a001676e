#!/bin/bash
# A/B of the working tree's library against libregcn_hip_head.so (tools/build_head_variant.py) on
# the config-5 headline, alternating, after the parity tests named in $TESTS (pytest -k)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ab}
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTFILES -k "$TESTS" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest.log
fi
HEADLIB=$GRAFT_REPO_ROOT/re-gcn_amd/regcn_amd/libregcn_hip_head.so
C="python -u bench.py --no-extras --no-scale --no-cpu-baseline --steps 10 --warmup 2"
for v in new head new head; do
  if [ $v = head ]; then export REGCN_HIP_LIB=$HEADLIB; else unset REGCN_HIP_LIB; fi
  timeout -k 10 300 $C > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || { echo "bench $v failed"; tail -20 gpurun_out/${TAG}_$v.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/${TAG}_$v.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$v', d['value'], d['ms_per_step'], ' '.join('%s %.1f' % (n.replace('regcn_', '')[:28], v['avg_us']) for n, v in k.items() if v['avg_us'] > 300))" | tee -a gpurun_out/${TAG}.txt
done
echo "all ok"
