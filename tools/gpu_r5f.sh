#!/bin/bash
# round 5: crel sweep; sharded tests with crel rank views; 8-wave phase kernels A/B (ICEWS14s); simulation
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
REGCN_CREL_EB=32 timeout -k 10 300 python -u tools/crelprobe.py --mins 0,512,1024,2048 > gpurun_out/r5f_crel32.log 2>&1 || { echo "crel32 failed"; tail -20 gpurun_out/r5f_crel32.log; exit 1; }
REGCN_CREL_EB=16 timeout -k 10 300 python -u tools/crelprobe.py --mins 512,2048 > gpurun_out/r5f_crel16.log 2>&1 || { echo "crel16 failed"; tail -20 gpurun_out/r5f_crel16.log; exit 1; }
echo "crel sweep ok"
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "crel_gather" > gpurun_out/r5f_pytest1.log 2>&1 || { echo "pytest1 failed"; tail -40 gpurun_out/r5f_pytest1.log; exit 1; }
tail -1 gpurun_out/r5f_pytest1.log
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_sharded.py > gpurun_out/r5f_pytest2.log 2>&1 || { echo "pytest2 failed"; tail -40 gpurun_out/r5f_pytest2.log; exit 1; }
tail -1 gpurun_out/r5f_pytest2.log
timeout -k 10 300 python -u bench.py --config icews14s_lgcn_roth --no-scale --no-cpu-baseline --steps 64 > gpurun_out/r5f_ic_w4.json 2> gpurun_out/r5f_ic_w4.err || { echo "ic w4 failed"; tail -20 gpurun_out/r5f_ic_w4.err; exit 1; }
REGCN_HIP_LIB=$GRAFT_REPO_ROOT/re-gcn_amd/regcn_amd/libregcn_hip_w8.so timeout -k 10 300 python -u bench.py --config icews14s_lgcn_roth --no-scale --no-cpu-baseline --steps 64 > gpurun_out/r5f_ic_w8.json 2> gpurun_out/r5f_ic_w8.err || { echo "ic w8 failed"; tail -20 gpurun_out/r5f_ic_w8.err; exit 1; }
echo "icews a/b ok"
REGCN_HIP_LIB=$GRAFT_REPO_ROOT/re-gcn_amd/regcn_amd/libregcn_hip_w8.so timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "phase or golden or shared_parameter or relation_gru" > gpurun_out/r5f_w8_pytest.log 2>&1
echo "w8 pytest rc=$?"; tail -1 gpurun_out/r5f_w8_pytest.log
timeout -k 10 300 python -u tools/simprobe.py --world 8 > gpurun_out/r5f_sim.json 2> gpurun_out/r5f_sim.err || { echo "sim failed"; tail -30 gpurun_out/r5f_sim.err; exit 1; }
echo "all ok"
