#!/bin/bash
# Round-6 quick check: selected GPU tests (-k pattern), then bench.py --gpus 2 over gloo (two
# ranks spawned by bench.py itself on the box's one GPU) and the default bench line.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-quick}
K=${2:-}
mkdir -p $OUT
cd $ROOT
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -k "$K" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -n 3 $OUT/tests_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${SPAWN2:-}" ]; then
  timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 --points '' --cpu-seconds 0 > $OUT/bench2_$TAG.json 2> $OUT/bench2_$TAG.err
  rc=$?; echo "bench --gpus 2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --cpu-seconds ${CPUS:-0} ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python - $OUT/bench_$TAG.json <<'PY'
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value",r["value"],"ms",r["ms_per_step"],"frac",r["roofline"]["frac"])
for p in r["points"]:
    print(p["snr_db"],p["ms_per_step"],[(k["name"][:30],k["ms"],k["codewords"]) for k in p["kernels"]])
PY
