#!/bin/bash
# round 3: 8-B syndrome-table slots (4 MiB table; 2 MiB at BCHK_TAB_MAXLOAD=0.8): parity,
# bench lines; read-pattern microbenchmark; per-request-size TCC counters of the bench call
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03k
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_timed_path.py tests/test_syndtab.py -x -q \
    --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1'.split('/')[-1], d['ms_per_step'], [(k['name'][:26], k['ms']) for k in d['kernels']]); [print(p['snr_db'], p['ms_per_step'], [k['ms'] for k in p['kernels']]) for p in d['points']]"; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
show $OUT/bench.json
BCHK_TAB_MAXLOAD=0.8 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bench_2mib.json 2>> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
show $OUT/bench_2mib.json
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
