#!/bin/bash
# Round 4: long-code parity subset, then BCH(255,139,31) lines (old library vs current).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r04g}
mkdir -p $OUT
cd $ROOT
timeout -k 10 120 python -u scripts/diag_r04_coop.py 8 4 4.0 128 > $OUT/${TAG}_diag4.log 2>&1; rc=$?; echo "diag t4 rc=$rc"; cat $OUT/${TAG}_diag4.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/diag_r04_coop.py 8 15 5.0 256 > $OUT/${TAG}_diag15.log 2>&1; rc=$?; echo "diag t15 rc=$rc"; cat $OUT/${TAG}_diag15.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "long_code or config5 or j15_matches_oracle" > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
: > $OUT/${TAG}_255.jsonl
for PT in "--snr 5 --J 15" "--snr 6 --J -1" "--snr 7 --J 15"; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 $PT --steps 3 --warmup 1 >> $OUT/${TAG}_255.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "[$PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
