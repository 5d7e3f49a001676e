#!/bin/bash
# dataset-size bench legs: concurrency x pool sweep (value only; no CPU baseline, no scale legs);
# LIBS="name:lib ..." (lib "-" = the in-tree build) alternates library builds per point, REPS times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in $(seq 1 ${REPS:-1}); do
for cfg in ${CFGS:-icews14s_lgcn_roth gdelt}; do
  for cp in ${SWEEP:-4:16 8:16 8:32 16:32 2:16}; do
  for spec in ${LIBS:-cur:-}; do
    name=${spec%%:*}; lib=${spec#*:}; [ "$lib" = "-" ] && lib=""
    c=${cp%:*}; p=${cp#*:}
    v=$(env ${lib:+REGCN_HIP_LIB=$GRAFT_REPO_ROOT/$lib} timeout -k 10 200 python bench.py --config $cfg --no-scale --no-cpu-baseline --concurrent $c --pool $p --steps 64 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || { echo "sweep $cfg $cp failed"; exit 1; }
    echo "$name $cfg concurrent=$c pool=$p $v"
  done
  done
done
done
