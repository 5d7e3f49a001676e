#!/bin/bash
# round 5: crel sweep at config 5 (per-layer launches) and the 8-rank simulation
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
REGCN_CREL_EB=32 timeout -k 10 300 python -u tools/crelprobe.py --mins 0,512,1024,2048,4096 > gpurun_out/r5g_crel32.log 2>&1 || { echo "crel32 failed"; tail -20 gpurun_out/r5g_crel32.log; exit 1; }
REGCN_CREL_EB=16 timeout -k 10 300 python -u tools/crelprobe.py --mins 512,2048 > gpurun_out/r5g_crel16.log 2>&1 || { echo "crel16 failed"; tail -20 gpurun_out/r5g_crel16.log; exit 1; }
echo "crel sweep ok"
timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5g_sim.json 2> gpurun_out/r5g_sim.err || { echo "sim failed"; tail -30 gpurun_out/r5g_sim.err; exit 1; }
echo "all ok"
