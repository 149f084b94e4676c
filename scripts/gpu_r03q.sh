#!/bin/bash
# round 3: analytic-tail enumeration timed by step phase (experiment build libbchk_anprof)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03q
mkdir -p $OUT
cd $R
BCHK_LIB=$R/polar-codes-with-bch-kernel_amd/lib/libbchk_anprof.so timeout -k 10 240 python -u scripts/an_diag.py 2 > $OUT/an_prof.jsonl 2> $OUT/an_prof.err || { tail $OUT/an_prof.err; exit 1; }
timeout -k 10 240 python -u scripts/an_diag.py 2 > $OUT/an_diag.jsonl 2> $OUT/an_diag.err || { tail $OUT/an_diag.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/an_prof.jsonl'):
    d=json.loads(l); print(d['snr'], d['mean'], d['total_p50_p90_p99_max']); print(d['prof_sum']); [print(x) for x in d['prof_slowest']]
"
echo done
