#!/bin/bash
# dense wgrad tests, isolated S1 weight-gradient A/B (tools/wgrad_ab.py), then the 3-class bench with
# RPC_DENSE_WGRAD=<value> for each value (interleaved, twice)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense_bev.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > $OUT/pytest.log 2>&1 && tail -2 $OUT/pytest.log &&
timeout -k 10 200 python -u tools/wgrad_ab.py > $OUT/wgrad_ab.log 2>&1 && cat $OUT/wgrad_ab.log
