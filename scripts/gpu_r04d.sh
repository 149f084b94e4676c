#!/bin/bash
# Round 4: BCH(255,139,31) at 5 dB J=15 and 6 dB J=inf over the search kernel's chunk limit
# (BCHK_CHUNK_LIMIT: chunks a codeword gets in the first pass before the cooperative kernel).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r04d}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}_255.jsonl
for LIMIT in ${LIMITS:-1 2 4 8}; do
  for PT in "--snr 5 --J 15" "--snr 6 --J -1"; do
    BCHK_CHUNK_LIMIT=$LIMIT timeout -k 10 200 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 $PT --steps 3 --warmup 1 > $OUT/${TAG}_tmp.json 2>> $OUT/${TAG}_255.err
    rc=$?; echo "[limit $LIMIT $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python -c "import json,sys; d=json.load(open('$OUT/${TAG}_tmp.json')); d['chunk_limit']=$LIMIT; print(json.dumps(d))" >> $OUT/${TAG}_255.jsonl
  done
done
