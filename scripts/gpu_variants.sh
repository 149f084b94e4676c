#!/bin/bash
# bench.py against experiment builds of libbchk (BCHK_LIB), a few workloads each.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-var}
shift
mkdir -p $OUT
cd $ROOT
: > $OUT/$TAG.jsonl
for V in "$@"; do
  for A in "--snr 5" "--snr 4" "--snr 5 --J -1"; do
    BCHK_LIB=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_$V.so timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 5 $A > $OUT/${TAG}_tmp.json 2>> $OUT/$TAG.err
    rc=$?; echo "[$V $A] rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 -c "import json,sys; d=json.loads(open('$OUT/${TAG}_tmp.json').read().strip().splitlines()[-1]); d['variant']='$V'; print(json.dumps(d))" >> $OUT/$TAG.jsonl
  done
done
