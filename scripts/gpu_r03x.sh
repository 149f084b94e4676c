#!/bin/bash
# round 3: first-pass cycles by phase (experiment build libbchk_anprof)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03x
mkdir -p $OUT
cd $R
BCHK_LIB=$R/polar-codes-with-bch-kernel_amd/lib/libbchk_anprof.so timeout -k 10 240 python -u scripts/an_diag.py 2 > $OUT/an_prof.jsonl 2> $OUT/an_prof.err || { tail $OUT/an_prof.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/an_prof.jsonl'):
    d=json.loads(l); fp=d['first_pass']; n=fp['codewords']; print(d['snr'], fp, {k: round(v/n) for k,v in fp.items()})
"
echo done
