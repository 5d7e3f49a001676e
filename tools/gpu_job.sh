#!/bin/bash
# The one GPU runner: JOBS="<job> <job> ..." TAG=<name> bash tools/gpu_job.sh
# Each job runs under its own time limit; the first failure ends the call (no retries).
#   tests        the whole -m gpu suite in one process, then smoke()
#   test:<expr>  pytest -m gpu -k <expr>
#   bench        the default bench line (N = 1)              -> gpurun_out/$TAG.bench.json
#   bench:<args> bench.py with <args> (commas for spaces)    -> gpurun_out/$TAG.bench.json
#   prof         kernel trace + stats of the short headline command
#   prof:<cfg>   kernel trace + stats of `bench.py --config <cfg>` (dataset sizes)
#   pmc          SQ / GRBM + L2-request / FETCH_SIZE / WRITE_SIZE passes of the short headline
#   agg[:uniform] the config-5 aggregation benchmark: kernel trace + FETCH / WRITE passes
#   simprof      kernel trace of the 8-rank owner-partition simulation (tools/simprobe.py)
#   py:<script>  python <script> (commas for spaces)         -> gpurun_out/$TAG.<n>.log
#   sh:<script>  bash <script> (commas for spaces)           -> gpurun_out/$TAG.<n>.log
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT/gpurun_out
TAG=${TAG:-job}
SHORT="python3 $GRAFT_REPO_ROOT/bench.py --no-extras --no-scale --no-cpu-baseline --steps 6 --warmup 1"
n=0
for job in $JOBS; do
  n=$((n + 1))
  arg=${job#*:}; arg=${arg//,/ }
  case "$job" in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $R/$TAG.pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $R/$TAG.pytest.log | head; tail -5 $R/$TAG.pytest.log; exit 1; }
      tail -1 $R/$TAG.pytest.log
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/$TAG.smoke.log 2>&1 || { echo "smoke failed"; tail -5 $R/$TAG.smoke.log; exit 1; } ;;
    test:*)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$arg" > $R/$TAG.$n.pytest.log 2>&1 || { echo "pytest -k $arg failed"; grep -E "FAILED|Error" $R/$TAG.$n.pytest.log | head; tail -5 $R/$TAG.$n.pytest.log; exit 1; }
      tail -1 $R/$TAG.$n.pytest.log ;;
    bench|bench:*)
      [ "$job" = bench ] && arg=""
      BENCH_DETAIL=$R/$TAG.$n.detail.json timeout -k 10 600 python -u bench.py $arg > $R/$TAG.$n.bench.json 2> $R/$TAG.$n.bench.err || { echo "bench $arg failed"; tail -20 $R/$TAG.$n.bench.err; exit 1; }
      tail -c 400 $R/$TAG.$n.bench.json ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$TAG.prof -o run -- $SHORT > $R/$TAG.prof.log 2>&1 || { echo "rocprof failed"; tail -5 $R/$TAG.prof.log; exit 1; } ;;
    prof:*)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$TAG.prof_$arg -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $arg --no-scale --no-cpu-baseline --steps 64 > $R/$TAG.prof_$arg.log 2>&1 || { echo "rocprof $arg failed"; tail -5 $R/$TAG.prof_$arg.log; exit 1; } ;;
    pmc)
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $R/$TAG.pmc_sq -o run -- $SHORT > $R/$TAG.pmc_sq.log 2>&1 || { echo "pmc sq failed"; exit 1; }
      timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT TCP_TCC_READ_REQ_sum --output-format csv -d $R/$TAG.pmc_grbm -o run -- $SHORT > $R/$TAG.pmc_grbm.log 2>&1 || { echo "pmc grbm failed"; exit 1; }
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$TAG.pmc_fetch -o run -- $SHORT > $R/$TAG.pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$TAG.pmc_write -o run -- $SHORT > $R/$TAG.pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
      python3 tools/pmc_summary.py $R/$TAG.pmc_sq $R/$TAG.pmc_grbm $R/$TAG.pmc_fetch $R/$TAG.pmc_write --match=k_rowtail,k_gather_agg,k_gather_crel,k_union_runs,k_score,k_gather_sum,k_init > $R/$TAG.pmc_summary.txt ;;
    agg|agg:uniform)
      # the config-5 aggregation benchmark: kernel trace + FETCH_SIZE / WRITE_SIZE (Zipf or uniform sources)
      u=""; t=agg; [ "$job" = agg:uniform ] && { u="--uniform-src"; t=agg_uniform; }
      A="python3 $GRAFT_REPO_ROOT/tools/aggbench.py --reps 2 --which union_aggregate,union_aggregate_src_runs,lorentz_aggregate $u"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$TAG.${t}_prof -o run -- $A > $R/$TAG.${t}_prof.log 2>&1 || { echo "agg rocprof failed"; exit 1; }
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$TAG.${t}_fetch -o run -- $A > $R/$TAG.${t}_fetch.log 2>&1 || { echo "agg pmc fetch failed"; exit 1; }
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$TAG.${t}_write -o run -- $A > $R/$TAG.${t}_write.log 2>&1 || { echo "agg pmc write failed"; exit 1; } ;;
    simprof)
      # kernel trace of the 8-rank owner-partition simulation, chunk tails on one stream (exclusive kernel times)
      REGCN_CHUNK_TAIL_STREAMS=1 timeout -k 10 420 rocprofv3 --kernel-trace -d $R/$TAG.simprof -o sim -- python3 $GRAFT_REPO_ROOT/tools/simprobe.py --world 8 > $R/$TAG.simprof.log 2>&1 || { echo "simprobe failed"; tail -20 $R/$TAG.simprof.log; exit 1; }
      python3 tools/simprof_summary.py $R/$TAG.simprof/sim_results.db --steps 6 --top 40 > $R/$TAG.simprof_summary.txt && rm -f $R/$TAG.simprof/sim_results.db ;;
    sh:*)
      timeout -k 10 900 bash $arg > $R/$TAG.$n.log 2>&1 || { echo "bash $arg failed"; tail -20 $R/$TAG.$n.log; exit 1; }
      tail -30 $R/$TAG.$n.log ;;
    py:*)
      timeout -k 10 600 python -u $arg > $R/$TAG.$n.log 2>&1 || { echo "python $arg failed"; tail -20 $R/$TAG.$n.log; exit 1; }
      tail -5 $R/$TAG.$n.log ;;
    *) echo "unknown job $job"; exit 2 ;;
  esac
  echo "[$job] ok"
done
echo "all ok"
