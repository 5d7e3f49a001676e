#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/graphdbg3.py > gpurun_out/graphdbg3.log 2>&1 || { echo "graphdbg3 failed"; tail -30 gpurun_out/graphdbg3.log; exit 1; }
grep -E "^key .*recorded|^graphs" gpurun_out/graphdbg3.log | cut -c1-1500
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sim_prof -o run -- python tools/simprobe.py --world 8 > gpurun_out/sim_prof.log 2>&1 || { echo "simprobe failed"; tail -20 gpurun_out/sim_prof.log; exit 1; }
grep "^{" gpurun_out/sim_prof.log | cut -c1-1500
bash tools/gpu_pmc_rowtail.sh
