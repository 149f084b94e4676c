#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run (no PMC counters).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-prof}
shift || true
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python3 $ROOT/bench.py --steps 5 --warmup 1 --cpu-seconds 0 "$@" > $OUT/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -h '^{' $OUT/prof_$TAG.log | cut -c1-400
cut -d, -f1-4 $OUT/prof_$TAG/run_kernel_stats.csv | head -8
exit $rc
