#!/bin/bash
# Round 4: long-code parity + lines (gpu_r04g.sh), then the cooperative kernel's cycle split:
# the same 5 dB J=15 and 6 dB J=inf lines with the split root test cut (libbchk_splitcut.so:
# Berlekamp-Massey alone, wrong results) and the diag build's per-codeword stamps.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r04m}
cd $ROOT
bash scripts/gpu_r04g.sh $TAG || exit 1
: > $OUT/${TAG}_splitcut.jsonl
for PT in "--snr 5 --J 15" "--snr 6 --J -1"; do
  BCHK_CUT_BUILD=1 BCHK_LIB=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_splitcut.so timeout -k 10 200 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 $PT --steps 3 --warmup 1 >> $OUT/${TAG}_splitcut.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "[splitcut $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
