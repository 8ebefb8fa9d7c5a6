#!/bin/bash
# CenterPoint e2e parity (conditioning-bounded), SECOND e2e backward-variant A/B, perf A/B, step profile
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_e2e_parity_centerpoint.py tests/test_gpu_perturber.py -v -s \
  --timeout 240 --timeout-method thread > $OUT/pytest_cp.log 2>&1; RC=$?
tail -3 $OUT/pytest_cp.log
[ $RC -ne 0 ] && [ $RC -ne 1 ] && exit $RC
bash tools/gpu_e2e_ab.sh $1 || exit $?
bash tools/gpu_ab_bench.sh $1 default RPC_PERT_SPLIT=0 RPC_SPARSE_FUSED_FIN=1 || exit $?
bash tools/gpu_bench_prof.sh $1
