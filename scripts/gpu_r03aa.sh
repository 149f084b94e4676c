#!/bin/bash
# round 3: long-code first kernel with the sent word prefetched; BCH(255) parity + configs;
# SC-list over the 64 x 64 eBCH kernel under rocprof
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03aa
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_timed_path.py -x -q \
    --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
run() { timeout -k 10 240 python bench.py --cpu-seconds 0 --points '' "$@" >> $OUT/cfg255.jsonl 2>> $OUT/cfg.err || exit 1; }
: > $OUT/cfg255.jsonl
for S in 6 7; do run --m 8 --t 15 --snr $S --J -1 --steps 3 --warmup 1; done
for S in 5 6 7; do run --m 8 --t 15 --snr $S --J 15 --steps 3 --warmup 1; done
python3 -c "
import json
for l in open('$OUT/cfg255.jsonl'):
    d=json.loads(l); print(d['config'].get('workload'), d['value'], d['ms_per_step'], [(k['name'][:30], k['ms']) for k in d['kernels']])
"
cd /tmp && export TMPDIR=/tmp
BENCH_B=2048 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ml -o run \
    -- python3 $R/scripts/bench_polar_ml.py > $OUT/polar_ml.jsonl 2> $OUT/polar_ml.err || { tail $OUT/polar_ml.err; exit 1; }
cat $OUT/polar_ml.jsonl | cut -c1-200
echo done
