#!/bin/bash
# round 3: fast kernel v2b (5-op keys, Green 16-sorter, read-back outputs) and the n <= 31
# uncapped analytic tail (an_osd): parity tests, BCH(31) J=inf timing, bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03g
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_timed_path.py -x -q \
    --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], [(k['name'][:26], k['ms']) for k in d['kernels']]); [print(p['snr_db'], p['ms_per_step'], [k['ms'] for k in p['kernels']]) for p in d['points']]"
for cfg in "5 3 -1 2.0" "5 3 -1 4.0" "5 3 15 2.0" "5 3 15 0.0"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --m $1 --t $2 --J $3 --snr $4 --points "" --batch 262144 --steps 10 --warmup 2 \
      --cpu-seconds 0 > $OUT/bench31_$1_$3_$4.json 2>> $OUT/bench.err || { echo "bench31 failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench31_$1_$3_$4.json').read().strip().splitlines()[-1]); print('BCH31', '$cfg', d['value'], d['ms_per_step'], [(k['name'][:26], k['ms'], k['codewords']) for k in d['kernels']])"
done
