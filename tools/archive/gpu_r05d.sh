#!/bin/bash
# r05: union GEMM microbenchmark on the metric's rulebooks; CenterPoint fp32 parity with mid-cell offsets
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/union_bench.py > $OUT/union_bench.log 2>&1; echo "union_bench rc $?"
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e_parity_centerpoint.py -v -s --timeout-method thread > $OUT/pytest_cp.log 2>&1; echo "cp rc $?"
tail -3 $OUT/pytest_cp.log
