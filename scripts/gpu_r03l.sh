#!/bin/bash
# round 3: where the fast kernel's extra read requests come from -- 128-B read requests per
# cut build (stage+keys / +sort / +prefix+S0 / +i=0 decode+accept / full) and per read pattern
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03l
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for n in 1 2 3 4 full; do
  if [ $n = full ]; then L=$R/polar-codes-with-bch-kernel_amd/lib/libbchk.so; else L=$R/polar-codes-with-bch-kernel_amd/lib/libbchk_cut$n.so; fi
  BCHK_LIB=$L timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum \
      -d $OUT/pmc_$n -o pmc --output-format csv -- python3 $R/scripts/fast_cut.py > $OUT/cut_$n.log 2>&1 || { tail $OUT/cut_$n.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum \
    -d $OUT/pmc_micro -o pmc --output-format csv -- $R/scripts/micro/load_patterns > $OUT/micro.log 2>&1 || { tail $OUT/micro.log; exit 1; }
echo done
