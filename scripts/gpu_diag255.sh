#!/bin/bash
# BCH(255,139,31) search-kernel diagnosis: SNR sweep, no-cooperative-kernel run, SQ counters.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-d255}
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}.jsonl
run() {
  timeout -k 10 200 python bench.py --cpu-seconds 0 --m 8 --t 15 --steps 3 --warmup 1 "$@" >> $OUT/${TAG}.jsonl 2>> $OUT/${TAG}.err
  rc=$?; echo "[$*] rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
for S in 6 7 8; do run --snr $S --J 15; done
BCHK_CHUNK_LIMIT=0 run --snr 7 --J 15
BCHK_CHUNK_LIMIT=0 run --snr 6 --J 15
cd /tmp && export TMPDIR=/tmp
for S in 6 7; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
     --kernel-trace --output-format csv -d $OUT/pmc_${TAG}_$S -o run \
     -- python3 $ROOT/bench.py --cpu-seconds 0 --m 8 --t 15 --steps 1 --warmup 0 --snr $S --J 15 > $OUT/pmc_${TAG}_$S.log 2>&1
  rc=$?; echo "pmc $S rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
