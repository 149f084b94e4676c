#!/bin/bash
# round 3: the ordered-statistics kernel LLRs (64 x 64 BCH kernel) and the mixed / Arikan
# SC-list decoders after the 64-bit row change
set -o pipefail
OUT=gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_polar_ml.py tests/test_polar_mixed.py tests/test_polar_sclist.py -x -v \
    --timeout 300 --timeout-method thread -m gpu > $OUT/polar_tests.log 2>&1
rc=$?
tail -25 $OUT/polar_tests.log
exit $rc
