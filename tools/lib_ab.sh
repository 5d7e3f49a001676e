#!/bin/bash
# A/B of library builds (and env variants) on the short config-5 headline, alternated REPS times
# on one box: each variant = a kernel trace + stats run (per-kernel averages) and a plain run
# (ms per step).  VARS="name:lib[:ENV=VAL] ..." (lib "-" = the in-tree build), REPS=2.
set -o pipefail
R=$GRAFT_REPO_ROOT/gpurun_out
TAG=${TAG:-ab}
REPS=${REPS:-2}
SHORT="python3 $GRAFT_REPO_ROOT/bench.py --no-extras --no-scale --no-cpu-baseline --steps 6 --warmup 1"
for r in $(seq 1 $REPS); do
  for spec in $VARS; do
    IFS=: read -r name lib env <<< "$spec"
    [ "$lib" = "-" ] && lib=""
    d=$R/$TAG.${name}_$r
    env ${lib:+REGCN_HIP_LIB=$GRAFT_REPO_ROOT/$lib} $env timeout -k 10 300 $SHORT > $d.json 2> $d.err || { echo "$name run $r failed"; tail -5 $d.err; exit 1; }
    ${lib:+export REGCN_HIP_LIB=$GRAFT_REPO_ROOT/$lib}
    [ -n "$env" ] && export "$env"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d.prof -o run -- $SHORT > $d.prof.log 2>&1 || { echo "$name rocprof $r failed"; exit 1; }
    unset REGCN_HIP_LIB; [ -n "$env" ] && unset "${env%%=*}"
    python3 $GRAFT_REPO_ROOT/tools/ab_summary.py $name $d.json $d.prof
  done
done
