#!/bin/bash
# Headline bench with different count_kernel grid caps (BCHK_COUNT_GRID).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-cgrid}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}.jsonl
for G in 16384 4096 2048 1024 512 256; do
  BCHK_COUNT_GRID=$G timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 20 >> $OUT/${TAG}.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "grid $G rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
for G in 16384 1024; do
  BCHK_COUNT_GRID=$G timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_$G -o run \
    -- python3 $ROOT/bench.py --cpu-seconds 0 --steps 5 > $OUT/prof_${TAG}_$G.log 2>&1
  rc=$?; echo "prof $G rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
