#!/bin/bash
# Config-5 entity-block work lists swept: WHICH=REL (relation means, REGCN_REL_BLOCK) or
# WHICH=HUB (hub pass, REGCN_HUB_BLOCK); 0 = plain chunks
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread > gpurun_out/rb_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/rb_pytest.log; exit 1; }
tail -3 gpurun_out/rb_pytest.log
for rb in ${BLOCKS:-0 1024 2048 4096}; do
export REGCN_${WHICH:-REL}_BLOCK=$rb
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/rb_bench_$rb.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/rb_bench_$rb.log; exit 1; }
python -c "import json,sys; j=json.loads([l for l in open('gpurun_out/rb_bench_$rb.log') if l.startswith('{')][-1]); k=j['kernels']; print('block=$rb', j['value'], j['ms_per_step'], k['regcn_segment_mean_f32']['avg_us'], k.get('regcn_union_aggregate_src_runs_f32', {}).get('avg_us'))"
done
