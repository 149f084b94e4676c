#!/bin/bash
# round 3: read-pattern microbenchmark for the fast kernel's rows; per-request-size TCC read
# counters (32/64/128-B requests) and write requests of the bench's call (fast_cut.py, full lib)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03j
mkdir -p $OUT
timeout -k 10 60 $R/scripts/micro/load_patterns > $OUT/load_patterns.jsonl 2>&1 || { cat $OUT/load_patterns.jsonl; exit 1; }
cat $OUT/load_patterns.jsonl
cd /tmp && export TMPDIR=/tmp
L=$R/polar-codes-with-bch-kernel_amd/lib/libbchk.so
BCHK_LIB=$L timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d $OUT/pmc_rd -o pmc --output-format csv -- python3 $R/scripts/fast_cut.py > $OUT/rd.log 2>&1 || { tail $OUT/rd.log; exit 1; }
BCHK_LIB=$L timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum \
    -d $OUT/pmc_wr -o pmc --output-format csv -- python3 $R/scripts/fast_cut.py > $OUT/wr.log 2>&1 || { tail $OUT/wr.log; exit 1; }
BCHK_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE \
    -d $OUT/pmc_fetch -o pmc --output-format csv -- python3 $R/scripts/fast_cut.py > $OUT/fetch.log 2>&1 || { tail $OUT/fetch.log; exit 1; }
echo done
