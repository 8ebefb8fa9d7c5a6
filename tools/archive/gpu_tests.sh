#!/bin/bash
# One gpurun call running selected GPU tests with output kept:
#   gpurun --timeout 900 -- bash tools/gpu_tests.sh <tag> <pytest args...>
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
RC=$?
tail -40 $OUT/pytest.log
exit $RC
