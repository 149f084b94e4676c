#!/bin/bash
# rocprofv3 kernel-trace summary of the BCH(255,139,31) configuration (BASELINE config 5 at 7 dB).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-p255}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python3 $ROOT/bench.py --cpu-seconds 0 --m 8 --t 15 --snr 7 --J 15 --steps 3 --warmup 1 > $OUT/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
