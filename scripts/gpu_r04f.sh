#!/bin/bash
# Round 4 A/B: the previous commit's library (libbchk_old.so) against the current one on
# BCH(255,139,31) 5 dB J=15 at 2^18 and 2^20 words; then the first kernel's phase cuts.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r04f}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}_ab.jsonl
for B in 262144 1048576; do
  for V in old new; do
    if [ $V = new ]; then L=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk.so; else L=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_old.so; fi
    BCHK_LIB=$L timeout -k 10 200 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 --snr 5 --J 15 --batch $B --steps 2 --warmup 1 > $OUT/${TAG}_tmp.json 2>> $OUT/${TAG}.err
    rc=$?; echo "[$V $B] rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python -c "import json; d=json.load(open('$OUT/${TAG}_tmp.json')); d['variant']='$V'; print(json.dumps(d))" >> $OUT/${TAG}_ab.jsonl
  done
done
bash scripts/gpu_first_cut.sh ${TAG}_fcut
