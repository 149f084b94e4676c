#!/bin/bash
# PMC counter passes (each in its own rocprofv3 run, --kernel-trace only beside --pmc)
# plus a chunk-limit sweep of the exact/cooperative hand-off. Stops at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0"
i=0
for CNT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/${TAG}_p$i -o run -- $BENCH > $OUT/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd $ROOT
[ "${PMC_NO_SWEEP:-0}" = 1 ] && exit 0
for CL in 0 2 4 8 16; do
  BCHK_CHUNK_LIMIT=$CL timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > $OUT/${TAG}_cl$CL.json 2>/dev/null
  rc=$?; echo "chunk_limit $CL rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
