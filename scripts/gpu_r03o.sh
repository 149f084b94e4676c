#!/bin/bash
# round 3: fast kernel, streamed row blocks vs 8-position slices (libbchk_slice.so): SQ
# instruction / wait counters per dispatch and HIP-event times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03o
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in slice stream; do
  if [ $v = stream ]; then L=$R/polar-codes-with-bch-kernel_amd/lib/libbchk.so; else L=$R/polar-codes-with-bch-kernel_amd/lib/libbchk_slice.so; fi
  BCHK_LIB=$L timeout -k 10 120 python3 $R/scripts/fast_cut.py > $OUT/time_$v.json 2>> $OUT/err.log || { echo "time $v failed"; exit 1; }
  echo "$v: $(cat $OUT/time_$v.json)"
  BCHK_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT \
      -d $OUT/pmc_$v -o pmc --output-format csv -- python3 $R/scripts/fast_cut.py >> $OUT/err.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo done
