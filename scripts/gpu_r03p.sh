#!/bin/bash
# round 3: fast kernel lockstep experiment -- the first round's second block per CU starts
# BCHK_FAST_STAGGER cycles late
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03p
mkdir -p $OUT
cd $R
for st in 0 10000 25000 50000 100000; do
  BCHK_FAST_STAGGER=$st timeout -k 10 120 python3 scripts/fast_cut.py > $OUT/time_$st.json 2>> $OUT/err.log || { echo "stagger $st failed"; exit 1; }
  echo "stagger $st: $(cat $OUT/time_$st.json)"
done
