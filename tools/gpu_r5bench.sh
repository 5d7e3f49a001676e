#!/bin/bash
# round 5: the default bench line alone
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u bench.py > gpurun_out/r5bench.json 2> gpurun_out/r5bench.err || { echo "bench failed"; tail -20 gpurun_out/r5bench.err; exit 1; }
tail -c 400 gpurun_out/r5bench.json
