#!/bin/bash
# round 5: per-workgroup stage stamps of the ICEWS14s phase launches (8-wave tiles)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/phasetrace.py > gpurun_out/r5n_phasetrace.log 2>&1 || { echo "phasetrace failed"; tail -20 gpurun_out/r5n_phasetrace.log; exit 1; }
cat gpurun_out/r5n_phasetrace.log | grep -v amdgpu.ids
