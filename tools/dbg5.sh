set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_training.py -v -s -x --timeout 300 --timeout-method thread -k "hip_graph or rejects" > gpurun_out/pt.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAIL" gpurun_out/pt.log | head -20; exit 1; }
grep -E "PASS|FAIL" gpurun_out/pt.log | cut -c1-120; tail -1 gpurun_out/pt.log
timeout -k 10 200 python tools/trainbench.py --no-cpu --graph > gpurun_out/tb.log 2>&1 || { echo "failed"; tail -30 gpurun_out/tb.log; exit 1; }
grep '^{' gpurun_out/tb.log | cut -c 190-
