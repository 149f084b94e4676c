#!/bin/bash
# Times the fast kernel cut after each phase (make -C polar-codes-with-bch-kernel_amd cuts).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
for n in 1 2 3 4 full; do
  if [ $n = full ]; then L=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk.so; else L=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_cut$n.so; fi
  BCHK_LIB=$L timeout -k 10 300 python scripts/fast_cut.py >> $OUT/fast_cut.jsonl 2>> $OUT/fast_cut.err
  rc=$?; echo "cut $n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
