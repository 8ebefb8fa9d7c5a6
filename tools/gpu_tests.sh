#!/bin/bash
# run selected GPU tests (args after the output tag are pytest node ids / -k expressions), then optionally a bench
#   tools/gpu_tests.sh TAG [BENCH=1] test_ids...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
BENCH=0
if [ "$1" = "BENCH=1" ]; then BENCH=1; shift; fi
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v -s --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ $BENCH = 1 ]; then
  timeout -k 10 400 python -u bench.py --steps 30 --warmup 10 > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-200
fi
