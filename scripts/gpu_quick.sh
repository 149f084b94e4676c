#!/bin/bash
# Quick GPU check: parity tests, then bench variants (env overrides), each under its own limit.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-quick}
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
shift || true
for V in "$@"; do
  env $V timeout -k 10 300 python bench.py --cpu-seconds 0 > $OUT/bench_${TAG}_${V//[ =]/_}.json 2>$OUT/bench_${TAG}.err
  rc=$?; echo "[$V] rc=$rc"; cat $OUT/bench_${TAG}_${V//[ =]/_}.json; [ $rc -eq 0 ] || exit $rc
done
