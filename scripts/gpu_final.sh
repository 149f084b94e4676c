#!/bin/bash
# Round artefacts: GPU parity tests, the default bench line (with the CPU baseline), a
# rocprofv3 kernel-trace summary of the same command, and the PMC HBM-traffic passes.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-final}
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 $OUT/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python3 $ROOT/bench.py --cpu-seconds 0 --points 5 > $OUT/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for CNT in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/traffic_${TAG}_p$i -o run \
      -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --points 5 > $OUT/traffic_${TAG}_p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($CNT) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $ROOT/scripts/pmc_summary.py $OUT/traffic_$TAG > $OUT/traffic_${TAG}_summary.json && echo summary ok
# bench.py's roofline `traffic` source: the headline workload's HBM bytes per launch
python3 $ROOT/scripts/traffic_json.py $OUT/traffic_${TAG}_summary.json 1048576 5.0 15 > $OUT/traffic_${TAG}.json \
    && echo traffic json ok
