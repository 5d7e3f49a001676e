#!/bin/bash
# round 5: 8-wave phase kernels (GRU parts wave-guarded) parity + ICEWS14s A/B; owner-sim kernel profile
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W8=$GRAFT_REPO_ROOT/re-gcn_amd/regcn_amd/libregcn_hip_w8.so
REGCN_HIP_LIB=$W8 timeout -k 10 150 python -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_gpu_parity.py -k "phase" > gpurun_out/r5h_w8_pytest.log 2>&1
rc=$?; echo "w8 pytest rc=$rc"; tail -1 gpurun_out/r5h_w8_pytest.log
[ $rc -le 1 ] || exit 1  # 1 = a failed assertion (not bitwise): still time it
timeout -k 10 150 python -u bench.py --config icews14s_lgcn_roth --no-scale --no-cpu-baseline --steps 64 > gpurun_out/r5h_ic_w4.json 2> gpurun_out/r5h_ic_w4.err || { echo "ic w4 failed"; tail -20 gpurun_out/r5h_ic_w4.err; exit 1; }
REGCN_HIP_LIB=$W8 timeout -k 10 150 python -u bench.py --config icews14s_lgcn_roth --no-scale --no-cpu-baseline --steps 64 > gpurun_out/r5h_ic_w8.json 2> gpurun_out/r5h_ic_w8.err || { echo "ic w8 failed"; tail -20 gpurun_out/r5h_ic_w8.err; exit 1; }
echo "icews a/b ok"
timeout -k 10 420 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/simprof6 -o sim -- python3 $GRAFT_REPO_ROOT/tools/simprobe.py --world 8 > gpurun_out/simprof6.log 2>&1 || { echo "simprof failed"; tail -20 gpurun_out/simprof6.log; exit 1; }
python3 tools/simprof_summary.py gpurun_out/simprof6/sim_results.db --top 60 > gpurun_out/simprof6_summary.txt && rm -f gpurun_out/simprof6/sim_results.db
echo "all ok"
