#!/bin/bash
# Round 4: a subset of the GPU tests (PYTEST_K), then the BCH(255,139,31) config-5 lines.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r04b}
mkdir -p $OUT
cd $ROOT
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$PYTEST_K" > $OUT/tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
: > $OUT/${TAG}_255.jsonl
run() {
  timeout -k 10 ${LIM:-200} python bench.py --cpu-seconds 0 --points '' "$@" >> $OUT/${TAG}_255.jsonl 2>> $OUT/${TAG}_255.err
  rc=$?; echo "[$*] rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run --m 8 --t 15 --snr 7 --J 15 --steps 3 --warmup 1
run --m 8 --t 15 --snr 6 --J -1 --steps 3 --warmup 1
run --m 8 --t 15 --snr 5 --J 15 --steps 3 --warmup 1
