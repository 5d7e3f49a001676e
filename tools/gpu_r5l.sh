#!/bin/bash
# round 5: rowtail.hip + score.hip without SLP vectorisation (no packed fp32 VALU beside MFMAs) A/B
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/re-gcn_amd/regcn_amd/libregcn_hip_noslp.so
C="python -u bench.py --no-extras --no-scale --no-cpu-baseline --steps 10 --warmup 2"
timeout -k 10 300 $C > gpurun_out/r5l_base.json 2> gpurun_out/r5l_base.err || { echo "base bench failed"; tail -20 gpurun_out/r5l_base.err; exit 1; }
REGCN_HIP_LIB=$V timeout -k 10 300 $C > gpurun_out/r5l_noslp.json 2> gpurun_out/r5l_noslp.err || { echo "noslp bench failed"; tail -20 gpurun_out/r5l_noslp.err; exit 1; }
timeout -k 10 300 $C > gpurun_out/r5l_base2.json 2> gpurun_out/r5l_base2.err || { echo "base2 bench failed"; tail -20 gpurun_out/r5l_base2.err; exit 1; }
REGCN_HIP_LIB=$V timeout -k 10 300 $C > gpurun_out/r5l_noslp2.json 2> gpurun_out/r5l_noslp2.err || { echo "noslp2 bench failed"; tail -20 gpurun_out/r5l_noslp2.err; exit 1; }
echo "all ok"
