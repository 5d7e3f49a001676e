#!/bin/bash
# round 5: what the owner-partition simulation's replicated time is made of (kernel trace with
# marker kernels around every simulated rank's launches, tools/sim_replicated.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
export REGCN_SIM_MARKERS=1
timeout -k 10 420 rocprofv3 --kernel-trace -d $R/gpurun_out/r5u_trace -o sim -- python3 $R/tools/simprobe.py --world 8 > $R/gpurun_out/r5u.log 2>&1 || { echo "simprobe failed"; tail -20 $R/gpurun_out/r5u.log; exit 1; }
python3 tools/sim_replicated.py gpurun_out/r5u_trace/sim_results.db --steps 3 > gpurun_out/r5u_replicated.txt && rm -f gpurun_out/r5u_trace/sim_results.db
head -45 gpurun_out/r5u_replicated.txt
