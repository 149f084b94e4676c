#!/bin/bash
# bench.py over the BASELINE.json configurations (one JSON line each, no CPU leg).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-cfg}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}.jsonl
run() {  # each configuration at its own Eb/N0 only (--points ''): the 4/5/6 dB curve is the headline's
  timeout -k 10 240 python bench.py --cpu-seconds 0 --points '' "$@" >> $OUT/${TAG}.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "[$*] rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
[ "${ONLY_LONG:-0}" = 1 ] || {
for S in 4 5 6; do run --snr $S; done
for S in 5 6; do run --snr $S --J -1; done
for S in 0 2 4 6; do run --m 5 --t 3 --batch 262144 --snr $S --J 15 --steps 5; done
for S in 2 4 6; do run --m 5 --t 3 --batch 262144 --snr $S --J -1 --steps 5; done
}
for S in 6 7; do run --m 8 --t 15 --snr $S --J -1 --steps 3 --warmup 1; done
for S in 5 6 7; do run --m 8 --t 15 --snr $S --J 15 --steps 3 --warmup 1; done
