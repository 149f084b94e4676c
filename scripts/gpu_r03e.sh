#!/bin/bash
# round 3: (1) the sharded fun() sweep's per-rank host time at world 1 / 2 / 4 (one generation
# thread per rank, so CPU seconds = host work), BCH(31,16,7) J=15, p=10^7, e=1000, and the
# reference md5 of p=10^6 e=100 at world 1 over RCCL; (2) SC-list over the 64 x 64 BCH kernel:
# bench + rocprof kernel stats
set -o pipefail
OUT=gpurun_out/r03e
mkdir -p $OUT
SD=polar-codes-with-bch-kernel_amd/sweep_dist.py
run() {  # name nproc backend p e extra
    BCHK_GEN_THREADS=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $2 \
        --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) $SD 5 3 $4 $5 --J 15 --backend $3 \
        --out $OUT/sweep_$1.csv $6 > $OUT/sweep_$1.log 2>&1 || { tail -20 $OUT/sweep_$1.log; return 1; }
    echo "$1 $(md5sum < $OUT/sweep_$1.csv | cut -c1-32) $(grep host_cpu_s $OUT/sweep_$1.log)"
}
run ref_w1_nccl 1 nccl 1000000 100 && run big_w1 1 gloo 10000000 1000 && run big_w2 2 gloo 10000000 1000 && \
  run big_w4 4 gloo 10000000 1000 && run big_w2_noresync 2 gloo 10000000 1000 --no-resync || exit 1
timeout -k 10 600 python -u scripts/bench_polar_ml.py > $OUT/polar_ml_bench.jsonl 2> $OUT/polar_ml_bench.err || { tail $OUT/polar_ml_bench.err; exit 1; }
cat $OUT/polar_ml_bench.jsonl
cd /tmp && export TMPDIR=/tmp
BENCH_B=4096 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_ml -o ml \
    -- python3 $GRAFT_REPO_ROOT/scripts/bench_polar_ml.py > $GRAFT_REPO_ROOT/$OUT/prof_ml.log 2>&1 || echo "rocprof rc=$?"
find $GRAFT_REPO_ROOT/$OUT/prof_ml -name "*stats*" | head
