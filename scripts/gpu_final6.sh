#!/bin/bash
# Round-6 artefacts: all GPU tests, the default bench line (CPU baseline), rocprofv3 kernel
# stats and memory-side traffic (PMC requests by size) of the headline; optionally (CONFIG5=1) config 5's lines with
# their PMC traffic and CPU baseline. Every GPU step under its own limit; stops at a failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-final6}
mkdir -p $OUT
cd $ROOT
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -n 2 $OUT/tests_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
pmc() {  # name, bench args: memory-side requests by size (reads, then writes), each pass its own run
  local nm=$1; shift
  local i=0
  for CNT in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
             "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/traffic_${nm}_p$i -o run \
        -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --points '' "$@" > $OUT/traffic_${nm}_p$i.log 2>&1
    rc=$?; echo "pmc $nm pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
( cd /tmp && export TMPDIR=/tmp && pmc $TAG --snr 5 ) || exit 1
python3 $ROOT/scripts/traffic_req_json.py $OUT/traffic_${TAG}_p1/run_counter_collection.csv $OUT/traffic_${TAG}_p2/run_counter_collection.csv 1048576 5.0 15 > $OUT/traffic_${TAG}.json && echo traffic json ok
timeout -k 10 300 python bench.py --traffic $OUT/traffic_${TAG}.json > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python3 $ROOT/bench.py --cpu-seconds 0 --points 5 > $OUT/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $ROOT
# bench.py --gpus 2 without a launcher: it spawns its two ranks (gloo: both on the box's one GPU)
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 --points '' --cpu-seconds 0 > $OUT/bench2_$TAG.json 2> $OUT/bench2_$TAG.err
rc=$?; echo "bench --gpus 2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
[ -n "${CONFIG5:-}" ] || exit 0
: > $OUT/${TAG}_255.jsonl
for PT in "5 15" "6 -1" "7 15"; do
  set -- $PT
  nm=${TAG}_255_${1}dB
  ( cd /tmp && export TMPDIR=/tmp && pmc $nm --m 8 --t 15 --snr $1 --J $2 ) || exit 1
  python3 $ROOT/scripts/traffic_req_json.py $OUT/traffic_${nm}_p1/run_counter_collection.csv $OUT/traffic_${nm}_p2/run_counter_collection.csv 1048576 $1.0 $2 > $OUT/traffic_${nm}.json
  timeout -k 10 400 python bench.py --m 8 --t 15 --snr $1 --J $2 --points '' --steps 5 --warmup 1 --cpu-seconds 12 \
      --traffic $OUT/traffic_${nm}.json >> $OUT/${TAG}_255.jsonl 2>> $OUT/${TAG}_255.err
  rc=$?; echo "[255 $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
