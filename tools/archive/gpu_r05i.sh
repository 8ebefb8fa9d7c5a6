#!/bin/bash
# r05: fp32 sparse GEMM two-level sums: sparse parity tests, SECOND e2e, CenterPoint e2e
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse_layers.py tests/test_gpu_sparse_basicblock.py tests/test_gpu_sparse_pipe.py tests/test_gpu_e2e_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_sparse.log 2>&1; echo "sparse rc $?"; tail -2 $OUT/pytest_sparse.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e_parity_centerpoint.py -v -s --timeout-method thread > $OUT/pytest_cp.log 2>&1; echo "cp rc $?"
tail -3 $OUT/pytest_cp.log
