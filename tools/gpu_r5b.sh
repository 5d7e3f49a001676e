#!/bin/bash
# round 5: halo exchange (sharded tests + rank simulation) and the config-5 owner simulation
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_sharded.py > gpurun_out/r5b_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r5b_pytest.log; exit 1; }
tail -2 gpurun_out/r5b_pytest.log
timeout -k 10 420 python -u tools/simprobe.py --world 8 > gpurun_out/r5b_sim.json 2> gpurun_out/r5b_sim.err || { echo "simprobe failed"; tail -30 gpurun_out/r5b_sim.err; exit 1; }
echo "sim ok"
timeout -k 10 420 rocprofv3 --kernel-trace -d gpurun_out/simprof5b -o sim -- python3 tools/simprobe.py --world 8 > gpurun_out/simprof5b.log 2>&1 || { echo "simprof failed"; tail -20 gpurun_out/simprof5b.log; exit 1; }
python3 tools/simprof_summary.py gpurun_out/simprof5b/sim_results.db --top 60 --from 2 > gpurun_out/simprof5b_summary.txt && rm -f gpurun_out/simprof5b/sim_results.db
echo "all ok"
