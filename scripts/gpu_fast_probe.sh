#!/bin/bash
# Fast-kernel experiments (round 5): stage times of the decode call for the ring kernel's
# knobs, then SQ counter passes of the ring kernel. One JSON line per configuration into
# gpurun_out/TAG_probe.jsonl; every GPU step under its own time limit, the first failure ends it.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-probe}
shift || true
mkdir -p $OUT
cd $ROOT
: > $OUT/${TAG}_probe.jsonl
for cfg in "$@"; do
  ENVS=${cfg%%|*}; ARGS=${cfg#*|}
  timeout -k 10 200 env $ENVS python scripts/fast_probe.py $ARGS --tag "$ENVS" >> $OUT/${TAG}_probe.jsonl 2>> $OUT/${TAG}_probe.err
  rc=$?; echo "[$cfg] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
if [ -n "${REQ:-}" ]; then
  # memory-side requests by size (reads, then writes) of the decode call, per configuration
  cd /tmp && export TMPDIR=/tmp
  j=0
  for cfg in "$@"; do
    j=$((j+1)); ENVS=${cfg%%|*}; ARGS=${cfg#*|}
    i=0
    for CNT in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
               "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      timeout -s KILL 120 env $ENVS rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/${TAG}_req${j}_$i -o run \
          -- python3 $ROOT/scripts/fast_probe.py --steps 2 $ARGS > $OUT/${TAG}_req${j}_$i.log 2>&1
      rc=$?; echo "req cfg $j pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
  cd $ROOT
fi
if [ -n "${PMC:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  i=0
  for CNT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/${TAG}_sq$i -o run \
        -- python3 $ROOT/scripts/fast_probe.py --steps 2 $PMC > $OUT/${TAG}_sq$i.log 2>&1
    rc=$?; echo "sq pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
exit 0
