#!/bin/bash
# r05: union GEMM tests + bench/profile, CenterPoint fp32 parity (fixed bounds, two sizes)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_sparse_pipe.py -x -q --timeout 150 --timeout-method thread > $OUT/pytest_sparse.log 2>&1; RC=$?
tail -3 $OUT/pytest_sparse.log
[ $RC -ne 0 ] && exit $RC
bash tools/gpu_prof_model.sh $1/bench --steps 20 --warmup 5 --no-parity-mode || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e_parity_centerpoint.py -v -s --timeout-method thread > $OUT/pytest_cp.log 2>&1; echo "cp rc $?"
tail -3 $OUT/pytest_cp.log
