#!/bin/bash
# the tests added this round, one pytest process
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_config5_pin.py "tests/test_gpu_parity.py::test_euclid_model_vs_golden" \
  "tests/test_gpu_training.py::test_loss_batches_memory_dense_fp64" ${EXTRA_TESTS} > gpurun_out/pytest_new.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/pytest_new.log | tail -30
exit $rc
