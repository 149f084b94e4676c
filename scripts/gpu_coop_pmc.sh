#!/bin/bash
# SQ counters of the long-code kernels (config 5, BCH(255,139,31)): LDS instructions, bank
# conflicts, LDS-array cycles and issue stalls of the cooperative / first / search kernels,
# over a 2^17-word 5 dB J=15 batch (scripts/fast_probe.py --m 8 --t 15). Each pass its own run.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-coop_pmc}
ARGS=${2:---m 8 --t 15 --snr 5 --batch 131072}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for CNT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/${TAG}_sq$i -o run \
      -- python3 $ROOT/scripts/fast_probe.py --steps 1 $ARGS > $OUT/${TAG}_sq$i.log 2>&1
  rc=$?; echo "sq pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
