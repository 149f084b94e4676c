#!/bin/bash
# Round 6 iteration: selected GPU tests (-k), then stage-time probes of the decode call for
# the given configurations ("ENV|ARGS"), optionally the first-pass timeline (FPTRACE=1).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=$1; K=$2; shift 2
mkdir -p $OUT
cd $ROOT
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -n 3 $OUT/tests_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
bash scripts/gpu_fast_probe.sh $TAG "$@" || exit 1
python - $OUT/${TAG}_probe.jsonl <<'PY'
import json,sys
for l in open(sys.argv[1]):
    r=json.loads(l); print(r.get("tag"), r.get("snr_db"), r.get("ms_per_step"), r.get("stages_ms"))
PY
if [ -n "${FPTRACE:-}" ]; then
  timeout -k 10 200 env BCHK_LIB=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_fptrace.so python scripts/fp_trace.py 5 > $OUT/${TAG}_fptrace5.json 2> $OUT/${TAG}_fptrace5.err || exit 1
  python -c "import json;r=json.load(open('$OUT/${TAG}_fptrace5.json'));print({k:r[k] for k in ('span_us','phase_mean_us','end_us_p50_p90_p99_last')})"
fi
