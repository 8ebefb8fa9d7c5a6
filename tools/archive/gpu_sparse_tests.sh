#!/bin/bash
# sparse-encoder GPU tests (layers, encoder, basic block, native backward, prefetch) + one 3-class bench
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse_layers.py tests/test_gpu_sparse_encoder.py tests/test_gpu_sparse_basicblock.py tests/test_gpu_prefetch.py tests/test_gpu_e2e_parity.py -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 && tail -2 $OUT/pytest.log &&
timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-200
