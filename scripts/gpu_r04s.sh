#!/bin/bash
# Round 4: the long-code parity subset on the default build, then cooperative-kernel claim-size variants (libbchk_xc_G.so: G chunks per claim; ring
# and tail claims as default) at BCH(255,139,31) 5 dB
# J=15 and 6 dB J=inf, each first checked: coop rows == exact-only rows (diag_r04_coop.py).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r04s}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}_xr.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "long_code or config5 or j15_matches_oracle" > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 $OUT/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for V in ${VARIANTS:-xc_16 xc_4 default}; do
  LIB=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_$V.so
  [ $V = default ] && LIB=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk.so
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
