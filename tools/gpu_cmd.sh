#!/bin/bash
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
shift
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
RC=$?
tail -30 $OUT/pytest.log
exit $RC
