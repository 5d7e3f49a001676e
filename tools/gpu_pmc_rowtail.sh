#!/bin/bash
# PMC passes over the config-5 per-layer predict (tools/c5probe.py): L2-side requests, SQ
# wait / MFMA-busy cycles, LDS instruction counts, per kernel (k_rowtail / k_gather_agg / ...).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python tools/c5probe.py --modes layers --reps 1"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc_sq -o run -- $P > gpurun_out/pmc_sq.log 2>&1 || { echo "pmc sq failed"; tail -5 gpurun_out/pmc_sq.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format csv -d gpurun_out/pmc_lds -o run -- $P > gpurun_out/pmc_lds.log 2>&1 || { echo "pmc lds failed"; tail -5 gpurun_out/pmc_lds.log; }
timeout -s KILL 300 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/pmc_l2 -o run -- $P > gpurun_out/pmc_l2.log 2>&1 || { echo "pmc l2 failed"; tail -5 gpurun_out/pmc_l2.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_grbm -o run -- $P > gpurun_out/pmc_grbm.log 2>&1 || { echo "pmc grbm failed"; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_sq gpurun_out/pmc_lds gpurun_out/pmc_l2 gpurun_out/pmc_grbm --match=k_rowtail,k_gather_agg,k_union_runs,k_score
