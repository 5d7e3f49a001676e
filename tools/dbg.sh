set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pt_all.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt_all.log; exit 1; }
tail -1 gpurun_out/pt_all.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof -o run -- python tools/trainbench.py --no-cpu --graph --steps 40 > gpurun_out/tprof.log 2>&1 || { echo "failed"; tail -20 gpurun_out/tprof.log; exit 1; }
grep '^{' gpurun_out/tprof.log | cut -c 190-
