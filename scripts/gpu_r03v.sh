#!/bin/bash
# round 3: packed DP counts in the tail plan; chunk-limit sweep with the faster tail
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03v}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_timed_path.py -x -q \
    --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 240 python -u scripts/an_diag.py 2 > $OUT/an_diag.jsonl 2> $OUT/an_diag.err || { tail $OUT/an_diag.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/an_diag.jsonl'):
    d=json.loads(l); print(d['snr'], d['mean'], d['total_p50_p90_p99_max']); [print(x) for x in d['slowest'][:3]]
"
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1'.split('/')[-1], d['ms_per_step'], [(k['name'][:40], k['ms']) for k in d['kernels']]); [print(p['snr_db'], p['ms_per_step'], [k['ms'] for k in p['kernels']]) for p in d['points']]"; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
show $OUT/bench.json
for cl in ${CLS:-}; do
  BCHK_CHUNK_LIMIT=$cl timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bench_cl$cl.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
  show $OUT/bench_cl$cl.json
done
echo done
