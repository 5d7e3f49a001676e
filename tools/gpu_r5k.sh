#!/bin/bash
# round 5: 4-wave scorer shape (REGCN_SCORE_NW=4) parity + headline A/B; tail-written send blocks
# (rank-simulation test) and the 8-rank simulation
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
REGCN_SCORE_NW=4 timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_decoder_c5.py -k "score or rank or decoder or ce or candidate" > gpurun_out/r5k_nw4_pytest.log 2>&1 || { echo "nw4 pytest failed"; tail -30 gpurun_out/r5k_nw4_pytest.log; exit 1; }
tail -1 gpurun_out/r5k_nw4_pytest.log
timeout -k 10 400 $T tests/test_gpu_sharded.py -k "rank_simulation or gather_rows or world2" > gpurun_out/r5k_send_pytest.log 2>&1 || { echo "send pytest failed"; tail -30 gpurun_out/r5k_send_pytest.log; exit 1; }
tail -1 gpurun_out/r5k_send_pytest.log
C="python -u bench.py --no-extras --no-scale --no-cpu-baseline --steps 10 --warmup 2"
timeout -k 10 300 $C > gpurun_out/r5k_nw8.json 2> gpurun_out/r5k_nw8.err || { echo "nw8 bench failed"; tail -20 gpurun_out/r5k_nw8.err; exit 1; }
REGCN_SCORE_NW=4 timeout -k 10 300 $C > gpurun_out/r5k_nw4.json 2> gpurun_out/r5k_nw4.err || { echo "nw4 bench failed"; tail -20 gpurun_out/r5k_nw4.err; exit 1; }
echo "headline a/b ok"
timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5k_sim.json 2> gpurun_out/r5k_sim.err || { echo "sim failed"; tail -30 gpurun_out/r5k_sim.err; exit 1; }
echo "all ok"
