#!/bin/bash
# round 5: first-round start stagger of the 64-row tails (REGCN_RT_STAGGER2 / 3) A/B on the headline
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="python -u bench.py --no-extras --no-scale --no-cpu-baseline --steps 10 --warmup 2"
for cfg in "0 0" "22 9" "11 5" "33 14" "0 0"; do
  set -- $cfg
  REGCN_RT_STAGGER2=$1 REGCN_RT_STAGGER3=$2 timeout -k 10 300 $C > gpurun_out/r5m_$1_$2.json 2> gpurun_out/r5m_$1_$2.err || { echo "bench $cfg failed"; tail -20 gpurun_out/r5m_$1_$2.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/r5m_$1_$2.json').read().strip().splitlines()[-1]);k=d['kernels']
print('$1 $2', d['value'], d['ms_per_step'], 'rt2 %.1f rt3 %.1f' % (k['regcn_layer_rowtail_f32']['avg_us'], k['regcn_layer_rowtail_f32(step)']['avg_us']))" | tee -a gpurun_out/r5m.txt
done
echo "all ok"
