#!/bin/bash
# BASELINE config 5 (BCH(255,139,31), batch 2^20) and config 2 (BCH(31,16,7), 2^18, 0..6 dB)
# bench lines, one JSON line each, no CPU leg. Stops at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-c255}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}.jsonl
run() {
  timeout -k 10 ${LIM:-200} python bench.py --cpu-seconds 0 "$@" >> $OUT/${TAG}.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "[$*] rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
for S in 7 6; do run --m 8 --t 15 --snr $S --J -1 --steps 3 --warmup 1; done
for S in 7 6 5; do run --m 8 --t 15 --snr $S --J 15 --steps 3 --warmup 1; done
