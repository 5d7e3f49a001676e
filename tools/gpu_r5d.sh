#!/bin/bash
# round 5: crel gather (relation half as one MFMA product per big tile) parity + headline + profile
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "crel_gather or fused_rank" > gpurun_out/r5d_pytest1.log 2>&1 || { echo "pytest1 failed"; tail -40 gpurun_out/r5d_pytest1.log; exit 1; }
tail -1 gpurun_out/r5d_pytest1.log
timeout -k 10 700 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gpu_rowtail.py tests/test_gpu_config5_pin.py tests/test_gpu_decoder_c5.py > gpurun_out/r5d_pytest2.log 2>&1 || { echo "pytest2 failed"; tail -40 gpurun_out/r5d_pytest2.log; exit 1; }
tail -1 gpurun_out/r5d_pytest2.log
timeout -k 10 400 python -u bench.py --no-extras --no-scale --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r5d_bench.json 2> gpurun_out/r5d_bench.err || { echo "bench failed"; tail -30 gpurun_out/r5d_bench.err; exit 1; }
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5d_prof -o run -- python3 bench.py --no-extras --no-scale --no-cpu-baseline --sim-ranks 0 --steps 6 --warmup 1 > gpurun_out/r5d_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/r5d_prof.log; exit 1; }
echo "all ok"
