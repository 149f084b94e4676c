#!/bin/bash
# Times kaneko_first_kernel<8,15> cut after each phase (make -C polar-codes-with-bch-kernel_amd fcuts)
# at BCH(255,139,31), 7 dB, J = 15; one bench JSON line per build.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-fcut}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}.jsonl
for n in ${CUTS:-1 2 3 4 full}; do
  if [ $n = full ]; then L=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk.so; elif [ $n = seq1 ]; then L=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_seq1.so; else L=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_fcut$n.so; fi
  BCHK_CUT_BUILD=1 BCHK_LIB=$L timeout -k 10 200 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 --snr 7 --J 15 --steps 3 --warmup 1 >> $OUT/${TAG}.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "cut $n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
