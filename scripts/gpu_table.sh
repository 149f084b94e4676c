#!/bin/bash
# GPU parity tests, then bench lines with and without the syndrome decoding table.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
TAG=${1:-filt}
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 5 $OUT/tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
: > $OUT/bench_$TAG.jsonl
run() {
  timeout -k 10 300 env "$@" >> $OUT/bench_$TAG.jsonl 2>> $OUT/bench_$TAG.err
  rc=$?; echo "[$*] rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run python bench.py --cpu-seconds 0
run BCHK_NO_TABLE=1 python bench.py --cpu-seconds 0
run python bench.py --cpu-seconds 0 --snr 4
run python bench.py --cpu-seconds 0 --snr 6
run python bench.py --cpu-seconds 0 --snr 5 --J -1
run python bench.py --cpu-seconds 0 --m 5 --t 3 --batch 262144 --snr 2 --J 15 --steps 5
run python bench.py --cpu-seconds 0 --m 5 --t 3 --batch 262144 --snr 0 --J 15 --steps 5
