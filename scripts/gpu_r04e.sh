#!/bin/bash
# Round 4: cooperative-kernel wave-count variants (libbchk_cwN.so) on BCH(255,139,31): parity
# of each against the exact-only path (scripts/diag_r04_coop.py), then the 5 dB J=15 and
# 6 dB J=inf lines.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r04e}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}_255.jsonl
for V in ${VARIANTS:-cw8 cw12 base}; do
  if [ $V = base ]; then L=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk.so; else L=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_$V.so; fi
  BCHK_LIB=$L timeout -k 10 120 python -u scripts/diag_r04_coop.py 8 4 4.0 128 > $OUT/${TAG}_diag_$V.log 2>&1
  rc=$?; echo "[$V diag] rc=$rc"; grep -c "equal to exact-only: True" $OUT/${TAG}_diag_$V.log; [ $rc -eq 0 ] || exit $rc
  for PT in "--snr 5 --J 15" "--snr 6 --J -1"; do
    BCHK_LIB=$L timeout -k 10 200 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 $PT --steps 3 --warmup 1 > $OUT/${TAG}_tmp.json 2>> $OUT/${TAG}_255.err
    rc=$?; echo "[$V $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python -c "import json; d=json.load(open('$OUT/${TAG}_tmp.json')); d['variant']='$V'; print(json.dumps(d))" >> $OUT/${TAG}_255.jsonl
  done
done
