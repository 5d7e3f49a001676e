#!/bin/bash
# rocprofv3 kernel stats of the config-5 owner-partition rank simulation (8 ranks, 4 chunks)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/simprof -o sim -- python3 $R/tools/simprobe.py --world 8 > $R/gpurun_out/simprof.log 2>&1
