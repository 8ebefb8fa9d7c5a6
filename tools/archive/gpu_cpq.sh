#!/bin/bash
# quick CenterPoint check: sparse bf16 kernel tests + bench + profile: tools/gpu_cpq.sh <tag> [pytest -k expr]
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_kernels.py tests/test_gpu_sparse_pipe.py -x -q --timeout 240 --timeout-method thread ${2:+-k "$2"} > $OUT/pytest.log 2>&1; RC=$?
tail -3 $OUT/pytest.log
[ $RC -ne 0 ] && exit $RC
bash tools/gpu_prof_model.sh $1 --model centerpoint --steps 8 --warmup 3
