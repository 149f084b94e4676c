#!/bin/bash
# round 3: fast kernel with streamed row blocks (16-B pieces, element-parallel keys, LDS key
# ring): parity, bench line, read requests, per-cut times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03n
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_timed_path.py -x -q \
    --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1'.split('/')[-1], d['ms_per_step'], [(k['name'][:26], k['ms']) for k in d['kernels']]); [print(p['snr_db'], p['ms_per_step'], [k['ms'] for k in p['kernels']]) for p in d['points']]"; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
show $OUT/bench.json
for cfg in "2 0"; do
  set -- $cfg
  BCHK_FAST_PERSIST=$1 BCHK_FAST_STAGGER=$2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bench_p$1_s$2.json 2>> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
  show $OUT/bench_p$1_s$2.json
done
for n in 1 2 3 4; do
  BCHK_LIB=$R/polar-codes-with-bch-kernel_amd/lib/libbchk_cut$n.so timeout -k 10 120 python3 $R/scripts/fast_cut.py > $OUT/time_$n.json 2>> $OUT/cut.err || { echo "cut $n failed"; exit 1; }
  echo "cut $n: $(cat $OUT/time_$n.json)"
done
cd /tmp && export TMPDIR=/tmp
BCHK_LIB=$R/polar-codes-with-bch-kernel_amd/lib/libbchk.so timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum \
    -d $OUT/pmc_rd -o pmc --output-format csv -- python3 $R/scripts/fast_cut.py > $OUT/rd.log 2>&1 || { tail $OUT/rd.log; exit 1; }
echo done
