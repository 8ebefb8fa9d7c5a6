#!/bin/bash
# Same-box A/B of the in-tree library (A) against librpc_hip_ab.so (B, tools/build_ab_lib.sh) on one bench model,
# alternating A B A B: tools/gpu_ab_model.sh <tag> <model: voxelnet|strong|centerpoint> [steps]
set -o pipefail
OUT=gpurun_out/$1
M=$2
S=${3:-30}
mkdir -p $OUT
export TMPDIR=/tmp
B=$PWD/robustpointclouds_amd/_lib/librpc_hip_ab.so
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model $M --steps $S --warmup 6 --no-cpu-baseline --no-parity-mode > $OUT/a_$i.log 2>&1 || exit 1
  RPC_HIP_LIB=$B timeout -k 10 300 python -u bench.py --model $M --steps $S --warmup 6 --no-cpu-baseline --no-parity-mode > $OUT/b_$i.log 2>&1 || exit 1
done
for f in $OUT/a_*.log $OUT/b_*.log; do
  echo "$(basename $f) $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("perturber_roofline", {}).get("perturber_fwd", {}).get("avg_ms"), d.get("perturber_roofline", {}).get("perturber_bwd", {}).get("avg_ms"))')"
done
