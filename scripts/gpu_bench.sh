#!/bin/bash
# One GPU session: bench (default config) then a rocprofv3 kernel-trace of a short run.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r01}
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python3 $ROOT/bench.py --steps 5 --warmup 1 --cpu-seconds 0 > $OUT/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
