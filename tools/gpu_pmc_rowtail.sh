#!/bin/bash
# PMC passes over the config-5 per-layer predict (tools/c5probe.py): L2-side requests, then SQ
# wait / MFMA-busy cycles, per kernel (k_rowtail / k_gather_agg / k_layer).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python tools/c5probe.py --modes layers --reps 1"
timeout -s KILL 300 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/pmc_l2 -o run -- $P > gpurun_out/pmc_l2.log 2>&1 || { echo "pmc l2 failed"; tail -5 gpurun_out/pmc_l2.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc_sq -o run -- $P > gpurun_out/pmc_sq.log 2>&1 || { echo "pmc sq failed"; tail -5 gpurun_out/pmc_sq.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_grbm -o run -- $P > gpurun_out/pmc_grbm.log 2>&1 || { echo "pmc grbm failed"; exit 1; }
echo pmc ok
