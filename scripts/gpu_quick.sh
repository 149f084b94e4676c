#!/bin/bash
# GPU parity tests + bench + diagnostic stamps (no rocprof). Stops on GPU faults.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-quick}
mkdir -p $OUT
cd $ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --cpu-seconds 0 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/diag_fast.py > $OUT/diag_fast_$TAG.json 2> $OUT/diag_fast_$TAG.err
rc=$?; echo "diag_fast rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/diag_coop.py > $OUT/diag_coop_$TAG.json 2> $OUT/diag_coop_$TAG.err
echo "diag_coop rc=$?"
