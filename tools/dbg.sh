set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof -o run -- python tools/trainbench.py --no-cpu --graph --steps 40 > gpurun_out/tprof.log 2>&1 || { echo "failed"; tail -20 gpurun_out/tprof.log; exit 1; }
grep '^{' gpurun_out/tprof.log
