#!/bin/bash
# round 5: ping-pong scorer (REGCN_SCORE_PP=1) parity + headline A/B; ICEWS14s phase-launch stage
# stamps (8-wave tiles); the owner-partition chunk x stream sweep
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
REGCN_SCORE_PP=1 timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_decoder_c5.py -k "score or rank or decoder or ce or candidate" > gpurun_out/r5p_pp_pytest.log 2>&1 || { echo "pp pytest failed"; tail -30 gpurun_out/r5p_pp_pytest.log; exit 1; }
tail -1 gpurun_out/r5p_pp_pytest.log
C="python -u bench.py --no-extras --no-scale --no-cpu-baseline --steps 10 --warmup 2"
for pp in 0 1 0 1; do
  REGCN_SCORE_PP=$pp timeout -k 10 300 $C > gpurun_out/r5p_pp$pp.json 2> gpurun_out/r5p_pp$pp.err || { echo "bench pp=$pp failed"; tail -20 gpurun_out/r5p_pp$pp.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/r5p_pp$pp.json').read().strip().splitlines()[-1]);k=d['kernels']['regcn_hyp_score_jobs_f32']
print('pp=$pp', d['value'], d['ms_per_step'], 'score %.1f us frac %.4f' % (k['avg_us'], k['frac']))" | tee -a gpurun_out/r5p_pp.txt
done
timeout -k 10 200 python -u tools/phasetrace.py > gpurun_out/r5n_phasetrace.log 2>&1 || { echo "phasetrace failed"; tail -20 gpurun_out/r5n_phasetrace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5n_phasetrace.log | head -12
bash tools/gpu_r5o.sh
