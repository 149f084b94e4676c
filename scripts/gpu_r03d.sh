#!/bin/bash
# round 3: the fast kernel's instructions per phase (builds cut after each phase, `make cuts`):
# SQ instruction counters per dispatch (rocprofv3 --pmc, one pass per build) and HIP-event
# times; plus the TCC counter list for per-request-size read counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03d
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || echo "counter list rc=$?"
for n in 1 2 3 4 full; do
  if [ $n = full ]; then L=$R/polar-codes-with-bch-kernel_amd/lib/libbchk.so; else L=$R/polar-codes-with-bch-kernel_amd/lib/libbchk_cut$n.so; fi
  BCHK_LIB=$L timeout -k 10 120 python3 $R/scripts/fast_cut.py > $OUT/time_$n.json 2>> $OUT/err.log || { echo "time $n failed"; exit 1; }
  BCHK_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
      SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc_$n -o pmc --output-format csv \
      -- python3 $R/scripts/fast_cut.py >> $OUT/err.log 2>&1 || { echo "pmc $n failed"; exit 1; }
  echo "cut $n: $(cat $OUT/time_$n.json)"
done
