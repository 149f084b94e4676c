#!/bin/bash
# round 3, first GPU call: the timed path pinned to the oracle at the timed config (+ config 4's
# 2^23 batch), then the default bench line
set -o pipefail
OUT=gpurun_out/r03a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_timed_path.py -x -v -s --timeout 400 --timeout-method thread \
    > $OUT/timed.log 2>&1 || { echo "timed-path tests failed"; tail -30 $OUT/timed.log; exit 1; }
tail -12 $OUT/timed.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json | head -c 1500
