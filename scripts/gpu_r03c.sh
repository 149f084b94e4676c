#!/bin/bash
# round 3: Kaneko / drop-in / channel / multirank GPU tests after the stream-engine rewrite,
# then the sharded fun() sweep's per-rank host time at world 1 (RCCL) and world 2 (gloo on
# the box's one GPU), BCH(31,16,7) J=15 p=10^6 e=100 (reference md5 105c77e4...)
set -o pipefail
OUT=gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_channel.py \
    tests/test_multirank.py tests/test_abi.py tests/test_timed_path.py -x -v --timeout 300 --timeout-method thread -m gpu \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
SD=polar-codes-with-bch-kernel_amd/sweep_dist.py
run() {  # name nproc backend extra
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $2 --master-addr 127.0.0.1 \
        --master-port $((29500 + RANDOM % 1000)) $SD 5 3 1000000 100 --J 15 --backend $3 $4 \
        > $OUT/sweep_$1.csv 2> $OUT/sweep_$1.err || { tail -20 $OUT/sweep_$1.err; return 1; }
    echo "$1 $(md5sum < $OUT/sweep_$1.csv | cut -c1-32) $(grep host_cpu_s $OUT/sweep_$1.err)"
}
run w1_nccl 1 nccl && run w2_gloo 2 gloo && run w2_gloo_noresync 2 gloo --no-resync && run w1_gloo 1 gloo
timeout -k 10 400 python -u scripts/tail_inline_check.py > $OUT/tail_inline.jsonl 2> $OUT/tail_inline.err; echo "tail_inline rc=$?"; cat $OUT/tail_inline.jsonl
