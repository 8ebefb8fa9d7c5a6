#!/bin/bash
# the whole GPU suite (as the driver runs it), then optional bench / profile steps
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; RC=$?
tail -3 $OUT/pytest_gpu.log
exit $RC
