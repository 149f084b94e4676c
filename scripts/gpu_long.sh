#!/bin/bash
# Long-code (m >= 7) check: GPU parity tests, then the BCH(255,139,31) bench lines.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-long}
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "long_code or j15_matches or m8 or infile" > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "long tests rc=$rc"; tail -n 3 $OUT/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_255.sh c255_$TAG
