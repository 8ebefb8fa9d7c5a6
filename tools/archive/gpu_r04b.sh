#!/bin/bash
# round 4: sparse mask-perm tests (gate the bench), fp32 CenterPoint parity-mode tests, then the SECOND
# bench + kernel trace
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_pipe.py tests/test_gpu_sparse_layers.py \
  tests/test_gpu_sparse_encoder.py tests/test_gpu_perturber.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; RC=$?
tail -3 $OUT/pytest.log
[ $RC -ne 0 ] && exit $RC
timeout -k 10 500 python -u -m pytest tests/test_gpu_dcn_head.py tests/test_gpu_centerpoint.py \
  tests/test_gpu_e2e_parity_centerpoint.py -v -s --timeout 240 --timeout-method thread > $OUT/pytest_cp.log 2>&1; RC=$?
tail -3 $OUT/pytest_cp.log
# assertion failures (1) still allow the bench; a timeout / crash / fault ends the call here
[ $RC -ne 0 ] && [ $RC -ne 1 ] && exit $RC
bash tools/gpu_ab_bench.sh $1 default RPC_SPARSE_PERM=0 RPC_SPARSE_FUSED_FIN=1 RPC_PERT_SPLIT=0 && \
bash tools/gpu_bench_prof.sh $1
