#!/bin/bash
# SC-list decoder throughput over a few codes and list sizes, then a rocprofv3 kernel
# summary of the main configuration.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-polar}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}_bench.jsonl
for cfg in "--n 10 --K 512 --L 8 --snr 2.0" "--n 10 --K 512 --L 8 --snr 3.0" "--n 10 --K 512 --L 1 --snr 2.0" \
           "--n 10 --K 512 --L 16 --snr 2.0 --batch 32768" "--n 8 --K 128 --L 32 --snr 2.0" \
           "--n 6 --K 32 --L 8 --snr 2.0 --batch 262144" "--n 11 --K 1024 --L 8 --snr 2.0 --batch 32768"; do
  timeout -k 10 200 python -u scripts/bench_polar.py $cfg --cpu-seconds 3 >> $OUT/${TAG}_bench.jsonl 2>> $OUT/${TAG}_bench.err
  rc=$?; echo "bench [$cfg] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python3 $ROOT/scripts/bench_polar.py --cpu-seconds 0 > $OUT/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
