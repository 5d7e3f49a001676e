#!/bin/bash
# round 5: multi-range fused rank count, two-stream chunk tails; simulation variants; headline budget sweep
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py::test_fused_rank_count_matches_score_matrix tests/test_gpu_decoder_c5.py tests/test_gpu_sharded.py > gpurun_out/r5c_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r5c_pytest.log; exit 1; }
tail -2 gpurun_out/r5c_pytest.log
timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5c_sim_default.json 2> gpurun_out/r5c_sim_default.err || { echo "sim default failed"; tail -30 gpurun_out/r5c_sim_default.err; exit 1; }
REGCN_RT_RG2_MIN_ROWS=16384 timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5c_sim_rg2.json 2> gpurun_out/r5c_sim_rg2.err || { echo "sim rg2 failed"; tail -30 gpurun_out/r5c_sim_rg2.err; exit 1; }
REGCN_CHUNK_TAIL_STREAMS=1 timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5c_sim_1stream.json 2> gpurun_out/r5c_sim_1stream.err || { echo "sim 1stream failed"; tail -30 gpurun_out/r5c_sim_1stream.err; exit 1; }
timeout -k 10 300 python -u tools/simprobe.py --world 8 --chunks 2 > gpurun_out/r5c_sim_c2.json 2> gpurun_out/r5c_sim_c2.err || { echo "sim c2 failed"; tail -30 gpurun_out/r5c_sim_c2.err; exit 1; }
echo "sims ok"
timeout -k 10 500 python -u tools/c5probe.py --modes layers --budgets 1024,2048,4096 --reps 5 > gpurun_out/r5c_budget.log 2>&1 || { echo "budget sweep failed"; tail -30 gpurun_out/r5c_budget.log; exit 1; }
echo "all ok"
