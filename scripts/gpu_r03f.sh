#!/bin/bash
# round 3: (1) ordered-statistics search v2 (fixed-disagreement bound, 12-B nodes): GPU tests,
# bench + rocprof; (2) fast kernel v2 (5-op sort keys, Green's 16-sorter): parity + timed-path
# tests, bench line; (3) sharded sweep md5 at world 2 / 4 after the global part decision
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03f
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_polar_ml.py tests/test_timed_path.py tests/test_gpu_parity.py -x -q \
    --timeout 300 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
head -c 900 $OUT/bench.json; echo
SD=polar-codes-with-bch-kernel_amd/sweep_dist.py
for w in 2 4; do
  BCHK_GEN_THREADS=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w \
      --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) $SD 5 3 10000000 1000 --J 15 --backend gloo \
      --out $OUT/sweep_big_w$w.csv > $OUT/sweep_big_w$w.log 2>&1 || { tail -20 $OUT/sweep_big_w$w.log; exit 1; }
  echo "w$w $(md5sum < $OUT/sweep_big_w$w.csv | cut -c1-32) $(grep host_cpu_s $OUT/sweep_big_w$w.log)"
done
BENCH_B=8192 timeout -k 10 400 python -u scripts/bench_polar_ml.py > $OUT/polar_ml_bench.jsonl 2> $OUT/polar_ml_bench.err || { tail $OUT/polar_ml_bench.err; exit 1; }
cat $OUT/polar_ml_bench.jsonl
cd /tmp && export TMPDIR=/tmp
BENCH_B=2048 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_ml -o ml \
    -- python3 $R/scripts/bench_polar_ml.py > $OUT/prof_ml.log 2>&1 || echo "rocprof rc=$?"
find $OUT/prof_ml -name "*stats*" | head -3
