#!/bin/bash
# S1 conv kernels: dense-engine GPU tests, then an interleaved A/B of the S1 variants at the SECOND shapes
#   gpurun --timeout 600 -- bash tools/gpu_conv_ab.sh <tag> [variants]
set -o pipefail
TAG=$1
VARS=${2:-0,1,2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense_bev.py -x -v --timeout 120 --timeout-method thread \
    > $OUT/pytest.log 2>&1
RC=$?
tail -5 $OUT/pytest.log
[ $RC -ne 0 ] && exit $RC
timeout -k 10 200 python -u tools/conv_bench.py --variants $VARS > $OUT/conv_bench.log 2>&1
RC=$?
cat $OUT/conv_bench.log
exit $RC
