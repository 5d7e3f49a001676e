#!/bin/bash
# round 5 final: the whole GPU suite, smoke(), the default bench line, the headline kernel trace
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r5final_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/r5final_pytest.log | head; tail -5 gpurun_out/r5final_pytest.log; exit 1; }
tail -1 gpurun_out/r5final_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5final_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r5final_smoke.log; exit 1; }
tail -1 gpurun_out/r5final_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r5final_bench.json 2> gpurun_out/r5final_bench.err || { echo "bench failed"; tail -20 gpurun_out/r5final_bench.err; exit 1; }
tail -c 300 gpurun_out/r5final_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5final_prof -o run -- python3 bench.py --no-extras --no-scale --no-cpu-baseline --steps 6 --warmup 1 > gpurun_out/r5final_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/r5final_prof.log; exit 1; }
echo "all ok"
