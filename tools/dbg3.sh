set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_autograd.py tests/test_gpu_training.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for e in hyperbolic_uvrgcn lgcn; do
timeout -k 10 200 python tools/trainbench.py --no-cpu --graph --encoder $e > gpurun_out/tb.log 2>&1 || { echo "failed"; tail -30 gpurun_out/tb.log; exit 1; }
grep '^{' gpurun_out/tb.log | cut -c 60-90,190-
done
