#!/bin/bash
# rocprofv3 kernel trace of the config-5 owner-partition rank simulation (8 ranks), summarised on the box
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 420 rocprofv3 --kernel-trace -d $R/gpurun_out/simprof5 -o sim -- python3 $R/tools/simprobe.py --world 8 > $R/gpurun_out/simprof5.log 2>&1 || { echo "simprobe failed"; tail -20 $R/gpurun_out/simprof5.log; exit 1; }
python3 tools/simprof_summary.py gpurun_out/simprof5/sim_results.db --top 60 > gpurun_out/simprof5_summary.txt && rm -f gpurun_out/simprof5/sim_results.db
tail -2 gpurun_out/simprof5.log
