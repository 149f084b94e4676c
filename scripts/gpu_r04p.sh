#!/bin/bash
# Round 4: (1) the long-code first kernel at 3 waves/SIMD (libbchk_lfw3.so: 156 VGPRs, no
# spills) against the default build (4 waves/SIMD, 128 VGPRs, 14 spilled) at BCH(255,139,31)
# 7 and 5 dB, with its PMC WRITE_SIZE; (2) the N > 1 bench path: two ranks over gloo on the
# box's one GPU (log kept for profiles/); (3) cooperative-kernel ring variants.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-r04p}
mkdir -p $OUT
cd $ROOT
LFW=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_lfw3.so
: > $OUT/${TAG}_lfw.jsonl
for PT in "--snr 7 --J 15" "--snr 5 --J 15"; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 $PT --steps 5 --warmup 1 >> $OUT/${TAG}_lfw.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "[default $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  BCHK_LIB=$LFW timeout -k 10 200 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 $PT --steps 5 --warmup 1 >> $OUT/${TAG}_lfw.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "[lfw3 $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
(cd /tmp && export TMPDIR=/tmp && BCHK_LIB=$LFW timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/${TAG}_lfw_wr -o run \
    -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --points '' --m 8 --t 15 --snr 7 --J 15 > $OUT/${TAG}_lfw_wr.log 2>&1)
rc=$?; echo "pmc lfw3 WRITE_SIZE rc=$rc"; [ $rc -eq 0 ] || exit $rc
# (3) the cooperative kernel's ring: 256 slots (xring256), + claims of 4 chunks in the last
# 60 chunks below the bound (xring256t)
: > $OUT/${TAG}_ring.jsonl
for PT in "--snr 5 --J 15" "--snr 6 --J -1"; do
  for V in xring256 xring256t; do
    BCHK_LIB=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_$V.so timeout -k 10 200 python bench.py --cpu-seconds 0 --points '' --m 8 --t 15 $PT --steps 3 --warmup 1 >> $OUT/${TAG}_ring.jsonl 2>> $OUT/${TAG}.err
    rc=$?; echo "[$V $PT] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/${TAG}_2rank_gloo.log 2>&1
rc=$?; echo "2-rank gloo rc=$rc"; tail -n 3 $OUT/${TAG}_2rank_gloo.log; exit $rc
