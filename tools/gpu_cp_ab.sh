#!/bin/bash
# CenterPoint-only same-box A/B of the in-tree library (a) against librpc_hip_ab.so (b), alternating, plus the
# CenterPoint GPU tests on the in-tree library: tools/gpu_cp_ab.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
B=$PWD/robustpointclouds_amd/_lib/librpc_hip_ab.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_centerpoint.py > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/acp_$i.log 2>&1 || exit 1
  RPC_HIP_LIB=$B timeout -k 10 200 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/bcp_$i.log 2>&1 || exit 1
done
tail -n 1 $OUT/pytest.log
for f in $OUT/acp_*.log $OUT/bcp_*.log; do
  echo "$(basename $f) $(tail -n 1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_roofline"]["stages"]; print(d["value"], d["ms_per_step"], "sparse_fwd", s["sparse_fwd"]["avg_ms"], "sparse_bwd", s["sparse_bwd"]["avg_ms"])')"
done
