#!/bin/bash
# r05: parity tests with the encoder oracle on HIP's ReLU decisions
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse_layers.py tests/test_gpu_e2e_parity.py -q -s --timeout 300 --timeout-method thread > $OUT/pytest_second.log 2>&1; echo "second rc $?"; tail -2 $OUT/pytest_second.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e_parity_centerpoint.py -v -s --timeout-method thread > $OUT/pytest_cp.log 2>&1; echo "cp rc $?"
tail -3 $OUT/pytest_cp.log
