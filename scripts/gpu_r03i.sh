#!/bin/bash
# round 3: search kernel with one search_codeword call site (inlined: LDS via ds_*, no
# scratch): parity, bench line, tail diagnostics, inline-tail check
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03i
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_timed_path.py -x -q \
    --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], [(k['name'][:26], k['ms']) for k in d['kernels']]); [print(p['snr_db'], p['ms_per_step'], [k['ms'] for k in p['kernels']]) for p in d['points']]"
timeout -k 10 240 python -u scripts/an_diag.py 3 > $OUT/an_diag.jsonl 2> $OUT/an_diag.err || { tail $OUT/an_diag.err; exit 1; }
timeout -k 10 240 python -u scripts/tail_inline_check.py > $OUT/tail_inline.jsonl 2> $OUT/tail_inline.err || { tail $OUT/tail_inline.err; exit 1; }
cat $OUT/tail_inline.jsonl | cut -c1-300
