#!/bin/bash
# Round 4: the cooperative kernel's cycle split again with the default ring (256 slots, tail
# claims), diag build, BCH(255,139,31) 2^17 words at 5 dB J=15 and 6 dB J=inf.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r04r}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}_diag.jsonl
for PT in "5.0 15" "6.0 -1"; do
  set -- $PT
  timeout -k 10 170 python -u scripts/diag_coop.py 8 15 $1 $2 131072 >> $OUT/${TAG}_diag.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "[diag $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
