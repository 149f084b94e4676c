#!/bin/bash
# round 3: first pass without the Chien rows in LDS, compiled for 5-8 waves per SIMD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03ac
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_timed_path.py -x -q \
    --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1'.split('/')[-1], d['ms_per_step'], [(k['name'][:40], k['ms']) for k in d['kernels']]); [print(p['snr_db'], p['ms_per_step'], [k['ms'] for k in p['kernels']]) for p in d['points']]"; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
show $OUT/bench.json
for w in 5 7 8; do
  BCHK_LIB=$R/polar-codes-with-bch-kernel_amd/lib/libbchk_fwpe$w.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/bench_w$w.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
  show $OUT/bench_w$w.json
done
echo done
