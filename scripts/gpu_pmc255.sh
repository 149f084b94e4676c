#!/bin/bash
# SQ counters of the BCH(255,139,31) kernels (5 dB, J = 15, 2^18 codewords): instruction mix
# and where the wave cycles go, one rocprofv3 --pmc pass per counter group.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-pmc255}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--m 8 --t 15 --snr ${SNR:-5} --J ${JJ:-15} --batch ${BATCH:-262144} --steps 1 --warmup 1 --points '' --cpu-seconds 0"
i=0
for CNT in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"; do
  i=$((i+1))
  eval timeout -s KILL 150 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/${TAG}_p$i -o run \
      -- python3 $ROOT/bench.py $ARGS > $OUT/${TAG}_p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
