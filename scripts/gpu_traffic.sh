#!/bin/bash
# HBM traffic of every kernel from PMC counters: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes (each beside --kernel-trace only), then a per-kernel summary.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-traffic}
shift || true
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CNT in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/${TAG}_p$i -o run \
      -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0 "$@" > $OUT/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i ($CNT) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $ROOT/scripts/pmc_summary.py $OUT/$TAG > $OUT/${TAG}_summary.json && echo summary ok
