#!/bin/bash
# Round 6: f4 (SC-list over the 64 x 64 extended-BCH kernel) with time-budgeted launches --
# throughput at each budget (BUDGETS, ms; 0 = one launch per call), then the rocprofv3 kernel
# durations of a call at the first budget.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/f4
mkdir -p $OUT
cd $ROOT
: > $OUT/bench.jsonl
for b in ${BUDGETS:-10 0}; do
  timeout -k 10 300 env BCHK_POLAR_BUDGET_MS=$b python scripts/bench_polar_ml.py >> $OUT/bench.jsonl 2>> $OUT/bench.err
  rc=$?; echo "bench budget $b rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cat $OUT/bench.jsonl
cd /tmp && export TMPDIR=/tmp
b=$(echo ${BUDGETS:-10 0} | cut -d' ' -f1)
BCHK_POLAR_BUDGET_MS=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python3 $ROOT/scripts/bench_polar_ml.py > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
