#!/bin/bash
# r05: union GEMM (deep weight prefetch) tests + bench/profile, CenterPoint flip analysis
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_sparse_pipe.py -x -q --timeout 150 --timeout-method thread > $OUT/pytest_sparse.log 2>&1; RC=$?
tail -3 $OUT/pytest_sparse.log
[ $RC -ne 0 ] && exit $RC
bash tools/gpu_prof_model.sh $1/bench --steps 20 --warmup 5 --no-parity-mode || exit $?
timeout -k 10 600 python -u tools/dbg_cp_flip.py > $OUT/cp_flip.log 2>&1; echo "cp_flip rc $?"
