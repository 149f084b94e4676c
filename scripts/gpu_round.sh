#!/bin/bash
# One GPU session: GPU parity tests, bench, rocprofv3 kernel trace of a short bench.
# Stops at the first GPU fault/abort/timeout (rc >= 124 or signal); plain test failures
# (rc 1) still let the bench run so the numbers can be inspected.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-run}
BENCH_ARGS=${2:-}
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py $BENCH_ARGS > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_$TAG.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python3 $ROOT/bench.py --steps 5 --warmup 1 --cpu-seconds 0 $BENCH_ARGS > $OUT/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
