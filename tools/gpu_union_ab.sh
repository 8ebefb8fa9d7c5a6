#!/bin/bash
# A/B: sparse GEMM source-row unions on / off, KITTI 3-class and CenterPoint benches
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
for u in 0 1; do
  RPC_SPARSE_UNION=$u timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-parity-mode --no-cpu-baseline > $OUT/kitti_u$u.log 2>&1 || exit $?
  tail -1 $OUT/kitti_u$u.log | cut -c1-200
  RPC_SPARSE_UNION=$u timeout -k 10 300 python -u bench.py --model centerpoint --steps 10 --warmup 3 --no-parity-mode --no-cpu-baseline > $OUT/cp_u$u.log 2>&1 || exit $?
  tail -1 $OUT/cp_u$u.log | cut -c1-200
done
