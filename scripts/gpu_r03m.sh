#!/bin/bash
# round 3: quotient syndrome table (8-B slots, 4 MiB; 2 MiB at BCHK_TAB_MAXLOAD=0.8), first
# pass held to 5 waves/SIMD: parity, bench lines; then where the fast kernel's extra read
# requests come from (128-B read requests per cut build and per read pattern)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03m
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
cd /tmp && export TMPDIR=/tmp
for n in 1 2 3 4 full; do
  if [ $n = full ]; then L=$R/polar-codes-with-bch-kernel_amd/lib/libbchk.so; else L=$R/polar-codes-with-bch-kernel_amd/lib/libbchk_cut$n.so; fi
  BCHK_LIB=$L timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum \
      -d $OUT/pmc_$n -o pmc --output-format csv -- python3 $R/scripts/fast_cut.py > $OUT/cut_$n.log 2>&1 || { tail $OUT/cut_$n.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum \
    -d $OUT/pmc_micro -o pmc --output-format csv -- $R/scripts/micro/load_patterns > $OUT/micro.log 2>&1 || { tail $OUT/micro.log; exit 1; }
echo done
