#!/bin/bash
# round 5: the new parity tests (full-size dataset configs vs the oracle, the config-5 decoder vs
# float64, sharded + analysis, the RCCL device branches), the GDELT bench leg and a 2-rank gloo
# rehearsal of the dataset configs' edge-partition leg
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gpu_parity.py::test_fused_rank_count_matches_score_matrix tests/test_gpu_dataset_full.py tests/test_gpu_decoder_c5.py tests/test_gpu_sharded.py > gpurun_out/r5a_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r5a_pytest.log; exit 1; }
tail -3 gpurun_out/r5a_pytest.log
timeout -k 10 300 python -u bench.py --config gdelt --steps 32 > gpurun_out/r5a_gdelt.json 2> gpurun_out/r5a_gdelt.err || { echo "gdelt bench failed"; tail -20 gpurun_out/r5a_gdelt.err; exit 1; }
echo "gdelt bench ok"
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --config gdelt --gpus 2 --steps 16 > gpurun_out/r5a_gdelt_w2.json 2> gpurun_out/r5a_gdelt_w2.err || { echo "gdelt w2 failed"; tail -20 gpurun_out/r5a_gdelt_w2.err; exit 1; }
echo "all ok"
