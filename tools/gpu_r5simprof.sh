#!/bin/bash
# round 5: kernel trace of the 8-rank owner-partition simulation with the chunk tails on ONE stream
# (exclusive kernel times), summarised per kernel over the 6 steps after the warm-up
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
REGCN_CHUNK_TAIL_STREAMS=1 timeout -k 10 420 rocprofv3 --kernel-trace -d $R/gpurun_out/simprof7 -o sim -- python3 $R/tools/simprobe.py --world 8 > $R/gpurun_out/simprof7.log 2>&1 || { echo "simprobe failed"; tail -20 $R/gpurun_out/simprof7.log; exit 1; }
python3 tools/simprof_summary.py gpurun_out/simprof7/sim_results.db --steps 6 --top 40 > gpurun_out/simprof7_summary.txt && rm -f gpurun_out/simprof7/sim_results.db
head -30 gpurun_out/simprof7_summary.txt
