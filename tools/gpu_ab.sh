#!/bin/bash
# Same-box A/B of the in-tree library (A) against robustpointclouds_amd/_lib/librpc_hip_ab.so (B, see
# tools/build_ab_lib.sh), alternating A B A B on the 3-class and CenterPoint bench lines: tools/gpu_ab.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
B=$PWD/robustpointclouds_amd/_lib/librpc_hip_ab.so
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity-mode > $OUT/a3_$i.log 2>&1 || exit 1
  RPC_HIP_LIB=$B timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity-mode > $OUT/b3_$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/acp_$i.log 2>&1 || exit 1
  RPC_HIP_LIB=$B timeout -k 10 200 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/bcp_$i.log 2>&1 || exit 1
done
for f in $OUT/a3_*.log $OUT/b3_*.log $OUT/acp_*.log $OUT/bcp_*.log; do
  echo "$(basename $f) $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
