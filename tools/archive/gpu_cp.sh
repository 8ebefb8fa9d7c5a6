#!/bin/bash
# CenterPoint: head / e2e tests, then bench + profile
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dcn_head.py tests/test_gpu_centerpoint.py tests/test_gpu_center_head.py \
  tests/test_gpu_e2e_parity_centerpoint.py -x -v -s --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; RC=$?
tail -3 $OUT/pytest.log
[ $RC -ne 0 ] && exit $RC
bash tools/gpu_prof_model.sh $1 --model centerpoint --steps 8 --warmup 3
