#!/bin/bash
# One GPU session of the build -> measure loop (round 5 on):
#   scripts/gpu_check.sh TAG 'PYTEST_K' 'BENCH_ARGS;BENCH_ARGS;...' [rocprof]
# runs the GPU tests selected by -k PYTEST_K ('' = none, 'all' = the whole suite), then one
# bench.py line per ';'-separated argument set ('VAR=v ... | args' sets environment
# variables for that line) into gpurun_out/TAG_bench.jsonl, then (4th
# argument 'rocprof') a rocprofv3 kernel-trace summary of the first bench line. Every GPU
# step has its own time limit; the first failure ends the session.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=$1
SEL=${2:-}
BENCHES=${3:-}
PROF=${4:-}
mkdir -p $OUT
cd $ROOT
if [ -n "$SEL" ]; then
  if [ "$SEL" = all ]; then K=(); else K=(-k "$SEL"); fi
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      -p no:cacheprovider "${K[@]}" > $OUT/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" $OUT/${TAG}_tests.log | tail -n 3
  [ $rc -eq 0 ] || exit $rc
fi
: > $OUT/${TAG}_bench.jsonl
IFS=';' read -ra BL <<< "$BENCHES"
for b in "${BL[@]}"; do
  [ -n "${b// /}" ] || continue
  if [[ "$b" == *"|"* ]]; then ENVS=${b%%|*}; ARGS=${b#*|}; else ENVS=; ARGS=$b; fi
  timeout -k 10 400 env $ENVS python bench.py $ARGS >> $OUT/${TAG}_bench.jsonl 2>> $OUT/${TAG}_bench.err
  rc=$?; echo "bench [$b] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
if [ "$PROF" = rocprof ] && [ ${#BL[@]} -gt 0 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run \
      -- python3 $ROOT/bench.py --cpu-seconds 0 --points '' --steps 5 --warmup 1 ${BL[0]#*|} > $OUT/${TAG}_prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; exit $rc
fi
exit 0
