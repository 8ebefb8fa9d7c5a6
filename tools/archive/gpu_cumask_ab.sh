#!/bin/bash
# Side streams on a CU subset (RPC_SIDE_CUMASK = 2 / 4) vs every CU: CenterPoint and 3-class bench lines, alternating
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for m in 0 2 4; do
    RPC_SIDE_CUMASK=$m timeout -k 10 200 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/cp_m${m}_$i.log 2>&1 || exit 1
  done
done
for i in 1 2; do
  for m in 0 2 4; do
    RPC_SIDE_CUMASK=$m timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity-mode > $OUT/k3_m${m}_$i.log 2>&1 || exit 1
  done
done
for f in $OUT/cp_*.log $OUT/k3_*.log; do
  echo "$(basename $f) $(tail -n 1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_roofline"]["stages"]; print(d["value"], d["ms_per_step"], "sparse_fwd", s["sparse_fwd"]["avg_ms"], "sparse_bwd", s["sparse_bwd"]["avg_ms"])')"
done
