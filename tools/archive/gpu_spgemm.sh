#!/bin/bash
# sparse GEMM kernels: bit-identity / fused-finalize tests, the 64x64 timing arms, then the encoder A/B under a
# kernel trace
#   gpurun --timeout 900 -- bash tools/gpu_spgemm.sh <tag> [modes]
set -o pipefail
OUT=gpurun_out/$1
MODES=${2:-0,1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_pipe.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; RC=$?
tail -3 $OUT/pytest.log
[ $RC -ne 0 ] && exit $RC
timeout -k 10 200 python -u tools/spgemm_arms.py > $OUT/arms.log 2>&1; RC=$?
cat $OUT/arms.log
[ $RC -ne 0 ] && exit $RC
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u tools/spgemm_ab.py $MODES 20 > $OUT/ab.log 2>&1; RC=$?
grep mode $OUT/ab.log
find $OUT/prof -name '*.csv' -size +4M -delete 2>/dev/null
exit $RC
