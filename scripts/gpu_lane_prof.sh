#!/bin/bash
# Long-code lane pre-pass profile: rocprofv3 kernel stats of the decode call, then SQ counter
# passes, for the fast_probe.py arguments given (default: BCH(255,139,31), 7 dB, J = 15).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-lane}
shift || true
ARGS=${*:---m 8 --t 15 --snr 7}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o run \
    -- python3 $ROOT/scripts/fast_probe.py --steps 3 $ARGS > $OUT/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for CNT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/${TAG}_sq$i -o run \
      -- python3 $ROOT/scripts/fast_probe.py --steps 2 $ARGS > $OUT/${TAG}_sq$i.log 2>&1
  rc=$?; echo "sq pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
