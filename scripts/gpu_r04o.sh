#!/bin/bash
# Round 4: cooperative-kernel cycle split for BCH(255,139,31) (config 5).
#  1. diag build (libbchk_diag.so): per heavy codeword the acceptor's prep / wait / accept
#     cycles and the decoders' claim / wait cycles, 5 dB J=15 and 6 dB J=inf, 2^17 words;
#  2. the bench lines with the split root test cut (libbchk_splitcut.so: Berlekamp-Massey
#     alone, wrong results -- timing only) next to the full library's.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r04o}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}_diag.jsonl
for PT in "5.0 15" "6.0 -1"; do
  set -- $PT
  timeout -k 10 200 python -u scripts/diag_coop.py 8 15 $1 $2 131072 >> $OUT/${TAG}_diag.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "[diag $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
: > $OUT/${TAG}_split.jsonl
for PT in "--snr 5 --J 15" "--snr 6 --J -1"; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 $PT --steps 3 --warmup 1 >> $OUT/${TAG}_split.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "[full $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  BCHK_CUT_BUILD=1 BCHK_LIB=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_splitcut.so timeout -k 10 200 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 $PT --steps 3 --warmup 1 >> $OUT/${TAG}_split.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "[splitcut $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
