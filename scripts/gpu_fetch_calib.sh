#!/bin/bash
# FETCH_SIZE calibration (scripts/fetch_calib.hip): timing run, then one FETCH_SIZE pass.
# The binary is built on the CPU side first: make -C polar-codes-with-bch-kernel_amd fetch_calib
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
timeout -k 10 60 $ROOT/scripts/fetch_calib > $OUT/fetch_calib.log 2>&1
rc=$?; echo "calib rc=$rc"; cat $OUT/fetch_calib.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
    -d $OUT/fetch_calib_pmc -o run -- $ROOT/scripts/fetch_calib > $OUT/fetch_calib_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
