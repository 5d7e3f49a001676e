#!/bin/bash
# round 5: initial-state map (k_init_rows4: 16-B accesses, next row prefetched) vs k_rowmap, alternated;
# then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in 1 0 1 0; do
  REGCN_INIT_PLAIN=$p timeout -k 10 120 python -u tools/initbench.py >> gpurun_out/r5w.txt 2> gpurun_out/r5w.err || { echo "initbench failed"; tail -20 gpurun_out/r5w.err; exit 1; }
done
cat gpurun_out/r5w.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r5w_pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r5w_pytest.log | head; tail -5 gpurun_out/r5w_pytest.log; exit 1; }
tail -1 gpurun_out/r5w_pytest.log
echo "all ok"
