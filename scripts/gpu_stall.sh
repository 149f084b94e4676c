#!/bin/bash
# Stall breakdown (SQ counters, one rocprofv3 --pmc pass per program) of the headline step's
# kernels and of the SC-list kernel at (1024, 512), L = 8: where the wave cycles go
# (active issue / issue stalls incl. LDS / parked on memory or barriers) and LDS pressure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-stall}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CNT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/${TAG}_kaneko -o run \
    -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --points 5 > $OUT/${TAG}_kaneko.log 2>&1
rc=$?; echo "kaneko pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/${TAG}_polar -o run \
    -- python3 $ROOT/scripts/bench_polar.py --n 10 --K 512 --L 8 --snr 2.0 --batch 16384 --cpu-seconds 0 > $OUT/${TAG}_polar.log 2>&1
rc=$?; echo "polar pass rc=$rc"; exit $rc
