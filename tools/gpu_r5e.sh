#!/bin/bash
# round 5: crel sweep (threshold x loads in flight), sharded tests with crel rank views, simulation
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "crel_gather" > gpurun_out/r5e_pytest1.log 2>&1 || { echo "pytest1 failed"; tail -40 gpurun_out/r5e_pytest1.log; exit 1; }
tail -1 gpurun_out/r5e_pytest1.log
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_sharded.py > gpurun_out/r5e_pytest2.log 2>&1 || { echo "pytest2 failed"; tail -40 gpurun_out/r5e_pytest2.log; exit 1; }
tail -1 gpurun_out/r5e_pytest2.log
REGCN_CREL_EB=32 timeout -k 10 300 python -u tools/crelprobe.py --mins 0,512,1024,2048 > gpurun_out/r5e_crel32.log 2>&1 || { echo "crel32 failed"; tail -20 gpurun_out/r5e_crel32.log; exit 1; }
REGCN_CREL_EB=16 timeout -k 10 300 python -u tools/crelprobe.py --mins 512,2048 > gpurun_out/r5e_crel16.log 2>&1 || { echo "crel16 failed"; tail -20 gpurun_out/r5e_crel16.log; exit 1; }
echo "crel sweep ok"
timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5e_sim.json 2> gpurun_out/r5e_sim.err || { echo "sim failed"; tail -30 gpurun_out/r5e_sim.err; exit 1; }
echo "all ok"
