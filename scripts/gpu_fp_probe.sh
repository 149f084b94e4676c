#!/bin/bash
# Round 6: first-pass (n <= 63 exact kernel) probes -- persistent grids, per-phase cycles of
# the experiment build (BCHK_AN_PROF), SQ occupancy counters of the headline step.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-fp}
mkdir -p $OUT
cd $ROOT
timeout -k 10 60 env BCHK_VERBOSE=1 python -c "
import sys; sys.path.insert(0,'tests')
from bchk_pkg import load
F=load(); d=F.KanekoKernelProcessor(6,6,J=15); d8=F.KanekoKernelProcessor(8,15,J=15)" > $OUT/${TAG}_grid.log 2>&1
rc=$?; cat $OUT/${TAG}_grid.log | grep bchk; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 env BCHK_LIB=$ROOT/polar-codes-with-bch-kernel_amd/lib/libbchk_xanprof.so python scripts/an_diag.py 1 > $OUT/${TAG}_anprof.jsonl 2> $OUT/${TAG}_anprof.err
rc=$?; echo "anprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "
import json,sys
r=json.loads(open('$OUT/${TAG}_anprof.jsonl').read().splitlines()[-1]); fp=r['first_pass']
n=fp['codewords']; print('first pass per codeword', {k: round(v/n) for k,v in fp.items()})"
cd /tmp && export TMPDIR=/tmp
CNT="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d $OUT/${TAG}_sq1 -o run \
    -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --points '' > $OUT/${TAG}_sq1.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $ROOT
for k in kaneko_search_kernel kaneko_fast_ring; do echo "== $k"; python scripts/sq_summary.py $OUT/${TAG} $k; done
