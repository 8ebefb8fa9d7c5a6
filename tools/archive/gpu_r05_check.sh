#!/bin/bash
# r05: focused GPU tests + the 3-class and CenterPoint bench lines: tools/gpu_r05_check.sh <tag> <test files...>
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
RC=$?
tail -2 $OUT/pytest.log
[ $RC -eq 0 ] || exit $RC
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-200 &&
timeout -k 10 300 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/bench_cp.log 2>&1 && tail -1 $OUT/bench_cp.log | cut -c1-200
