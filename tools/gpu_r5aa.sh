#!/bin/bash
# round 5: crel minimum tile count default (768): the crel test and the headline (crel still on at config 5)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "crel" > gpurun_out/r5aa_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r5aa_pytest.log; exit 1; }
tail -1 gpurun_out/r5aa_pytest.log
timeout -k 10 300 python -u tools/crelprobe.py --mins 2048 --reps 3 > gpurun_out/r5aa_crel.log 2>&1 || { echo "crelprobe failed"; tail -20 gpurun_out/r5aa_crel.log; exit 1; }
grep -v amdgpu gpurun_out/r5aa_crel.log | head -3
REGCN_CREL_MIN_TILES=0 timeout -k 10 300 python -u tools/crelprobe.py --mins 2048 --reps 3 > gpurun_out/r5aa_crel0.log 2>&1 || { echo "crelprobe0 failed"; exit 1; }
grep -v amdgpu gpurun_out/r5aa_crel0.log | head -3
echo "all ok"
