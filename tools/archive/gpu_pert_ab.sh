#!/bin/bash
# Perturber A/B: GPU perturber tests on the in-tree library, then tools/pert_bench.py and the 3-class bench line
# alternating in-tree (a) / librpc_hip_ab.so (b): tools/gpu_pert_ab.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
B=$PWD/robustpointclouds_amd/_lib/librpc_hip_ab.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_perturber.py > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u tools/pert_bench.py 20000,40000,80000 > $OUT/pa_$i.txt 2>&1 || exit 1
  RPC_HIP_LIB=$B timeout -k 10 200 python -u tools/pert_bench.py 20000,40000,80000 > $OUT/pb_$i.txt 2>&1 || exit 1
done
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity-mode > $OUT/a3_$i.log 2>&1 || exit 1
  RPC_HIP_LIB=$B timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity-mode > $OUT/b3_$i.log 2>&1 || exit 1
done
tail -n 1 $OUT/pytest.log
for f in $OUT/a3_*.log $OUT/b3_*.log; do
  echo "$(basename $f) $(tail -n 1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_roofline"]["stages"]; print(d["value"], d["ms_per_step"], "pert_fwd", s["perturber_fwd"]["avg_ms"], "pert_bwd", s["perturber_bwd"]["avg_ms"])')"
done
