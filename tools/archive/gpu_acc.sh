#!/bin/bash
# perf-mode accuracy: the fp16-forward kernels, the per-layer sparse encoder table (fp32 / perf / perf with bf16
# forward operands) and the 6-step bf16-vs-fp32 training trajectory
#   gpurun --timeout 900 -- bash tools/gpu_acc.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_kernels.py tests/test_gpu_sparse_layers.py tests/test_gpu_bf16_trajectory.py \
    tests/test_gpu_sparse_pipe.py -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; RC=$?
grep -E "layer|input gradient|cosine|passed|failed|Error" $OUT/pytest.log | tail -60
exit $RC
