#!/bin/bash
# round 5: PMC passes (one counter group per run) of the short headline command
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="python3 $GRAFT_REPO_ROOT/bench.py --no-extras --no-scale --no-cpu-baseline --steps 3 --warmup 1"
R=$GRAFT_REPO_ROOT/gpurun_out
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $R/r5j_sq -o run -- $C > $R/r5j_sq.log 2>&1 || { echo "pmc sq failed"; tail -5 $R/r5j_sq.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TCP_TCC_READ_REQ_sum --output-format csv -d $R/r5j_grbm -o run -- $C > $R/r5j_grbm.log 2>&1 || { echo "pmc grbm failed"; tail -5 $R/r5j_grbm.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/r5j_fetch -o run -- $C > $R/r5j_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -5 $R/r5j_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/r5j_write -o run -- $C > $R/r5j_write.log 2>&1 || { echo "pmc write failed"; tail -5 $R/r5j_write.log; exit 1; }
python3 tools/pmc_summary.py $R/r5j_sq $R/r5j_grbm $R/r5j_fetch $R/r5j_write --match=k_rowtail,k_gather_agg,k_gather_crel,k_union_runs,k_score,k_gather_sum,k_rowmap > $R/r5j_summary.txt
echo "all ok"
