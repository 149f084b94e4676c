#!/bin/bash
# round 3: helper waves in the analytic tail kernel (exact chunks, shared enumeration): tail parity, diagnostics, bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03s}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_timed_path.py -x -q \
    --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 240 python -u scripts/an_diag.py 2 > $OUT/an_diag.jsonl 2> $OUT/an_diag.err || { tail $OUT/an_diag.err; exit 1; }
BCHK_LIB=$R/polar-codes-with-bch-kernel_amd/lib/libbchk_anprof.so timeout -k 10 240 python -u scripts/an_diag.py 1 > $OUT/an_prof.jsonl 2> $OUT/an_diag.err || { tail $OUT/an_diag.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/an_diag.jsonl'):
    d=json.loads(l); print(d['snr'], d['mean']['plan'], d['mean']['after'], d['total_p50_p90_p99_max']); [print(x) for x in d['slowest'][:4]]
for l in open('$OUT/an_prof.jsonl'):
    d=json.loads(l); print('prof', d['snr'], d['prof_sum']); [print(x) for x in d['prof_slowest'][:2]]
"
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1'.split('/')[-1], d['ms_per_step'], [(k['name'][:40], k['ms']) for k in d['kernels']]); [print(p['snr_db'], p['ms_per_step'], [k['ms'] for k in p['kernels']]) for p in d['points']]"; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
show $OUT/bench.json
BCHK_AN_HELP=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bench_nohelp.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
show $OUT/bench_nohelp.json
echo done
