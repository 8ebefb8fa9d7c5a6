#!/bin/bash
# quick GPU test run: tools/gpu_quick.sh <tag> <pytest args...>
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "$@" -v -s --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; RC=$?
tail -4 $OUT/pytest.log
exit $RC
