#!/bin/bash
# Selected GPU tests, then an A/B of one environment toggle (tools/gpu_ab_env.sh), in one call
#   gpurun --timeout 1100 -- bash tools/gpu_tests_ab.sh <tag> <VAR> <pytest args...>
set -o pipefail
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
RC=$?
tail -3 $OUT/pytest.log
[ $RC -ne 0 ] && exit $RC
bash tools/gpu_ab_env.sh $TAG $VAR
