#!/bin/bash
# e2e fp32 parity test under the backward variants (which change moved middle.11.gamma)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
for v in default "RPC_SPARSE_NATIVE=0" "RPC_DENSE_BNFUSE=0" "RPC_SPARSE_NATIVE=0 RPC_DENSE_BNFUSE=0"; do
  echo "== $v" >> $OUT/e2e.log
  if [ "$v" = default ]; then E=""; else E="$v"; fi
  env $E timeout -k 10 300 python -u -m pytest "tests/test_gpu_e2e_parity.py::test_adversarial_step_fp32_hip_matches_oracle[3]" -x -q -s --timeout 280 --timeout-method thread >> $OUT/e2e.log 2>&1 || exit 1
done
grep -E "^==|middle.11|passed|failed|hip mean" $OUT/e2e.log
