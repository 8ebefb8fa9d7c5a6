#!/bin/bash
# mask-ordered sparse GEMM rows: tests, then bench + kernel trace
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_pipe.py tests/test_gpu_sparse_layers.py tests/test_gpu_sparse_encoder.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; RC=$?
tail -3 $OUT/pytest.log
[ $RC -ne 0 ] && exit $RC
bash tools/gpu_bench_prof.sh $1
