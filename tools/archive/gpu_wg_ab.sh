#!/bin/bash
# Sparse weight-gradient kernel A/B: bf16 kernel tests on the in-tree library, then the standalone per-layer
# timing (tools/spwg_bench.py) of the in-tree library (A) and librpc_hip_ab.so (B) on both models.
#   tools/gpu_wg_ab.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
B=$PWD/robustpointclouds_amd/_lib/librpc_hip_ab.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bf16_kernels.py > $OUT/pytest.log 2>&1 || exit 1
for m in centerpoint voxelnet; do
  timeout -k 10 200 python -u tools/spwg_bench.py $m > $OUT/a_$m.log 2>&1 || exit 1
  RPC_HIP_LIB=$B timeout -k 10 200 python -u tools/spwg_bench.py $m > $OUT/b_$m.log 2>&1 || exit 1
done
tail -n 2 $OUT/pytest.log
for f in $OUT/a_*.log $OUT/b_*.log; do echo "$(basename $f) $(tail -n 1 $f)"; done
