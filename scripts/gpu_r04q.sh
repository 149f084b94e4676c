#!/bin/bash
# Round 4: cooperative-kernel ring size / tail-claim variants (libbchk_xr_S_T_C.so: S ring
# slots, claims of C chunks in the last T chunks below the bound) at BCH(255,139,31) 5 dB
# J=15 and 6 dB J=inf, each first checked: coop rows == exact-only rows (diag_r04_coop.py).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r04q}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}_xr.jsonl
for V in xr_256_120_4 xr_256_60_2 xr_384_60_4 xring256t; do
  LIB=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_$V.so
  for A in "8 15 5.0 256" "7 10 5.0 256" "8 4 4.0 128"; do
    BCHK_LIB=$LIB timeout -k 10 120 python -u scripts/diag_r04_coop.py $A > $OUT/${TAG}_${V}_diag.log 2>&1
    rc=$?; echo "[$V diag $A] rc=$rc $(grep -c 'equal to exact-only: True' $OUT/${TAG}_${V}_diag.log) equal"; [ $rc -eq 0 ] || exit $rc
    grep -q "equal to exact-only: False" $OUT/${TAG}_${V}_diag.log && { echo "$V MISMATCH"; exit 1; }
  done
  for PT in "--snr 5 --J 15" "--snr 6 --J -1"; do
    BCHK_LIB=$LIB timeout -k 10 170 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 $PT --steps 3 --warmup 1 >> $OUT/${TAG}_xr.jsonl 2>> $OUT/${TAG}.err
    rc=$?; echo "[$V $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
