#!/bin/bash
# graph-replay drift diagnostics, the 8-rank owner simulation (chunk sweep), PMC passes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/graphdbg3.py > gpurun_out/graphdbg3.log 2>&1 || { echo "graphdbg3 failed"; tail -30 gpurun_out/graphdbg3.log; exit 1; }
grep -E "^key .*recorded|^graphs" gpurun_out/graphdbg3.log | cut -c1-1500
for c in 1 2 4; do
  timeout -k 10 300 python tools/simprobe.py --world 8 --chunks $c > gpurun_out/sim_c$c.log 2>&1 || { echo "simprobe $c failed"; tail -20 gpurun_out/sim_c$c.log; exit 1; }
  echo "chunks=$c $(grep '^{' gpurun_out/sim_c$c.log | cut -c1-700)"
done
bash tools/gpu_pmc_rowtail.sh
