#!/bin/bash
# Occupancy probe of the SC-list kernel: the default grid and explicit grids.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT; cd $ROOT
: > $OUT/grid.jsonl
export BCHK_POLAR_DEBUG=1
for L in 1 8; do
  for G in "" 256 512 1024 2048 4096; do
    if [ -n "$G" ]; then export BCHK_POLAR_GRID=$G; else unset BCHK_POLAR_GRID; fi
    echo "L=$L G=$G" >> $OUT/grid.jsonl
    timeout -k 10 120 python -u scripts/bench_polar.py --n 10 --K 512 --L $L --batch 32768 --steps 3 --cpu-seconds 0 >> $OUT/grid.jsonl 2>> $OUT/grid.err
    rc=$?; [ $rc -eq 0 ] || exit $rc
  done
done
