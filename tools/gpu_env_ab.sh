#!/bin/bash
# Same-box A/B of one environment switch on the 3-class and CenterPoint bench lines, alternating:
#   tools/gpu_env_ab.sh <tag> "VAR=value [VAR2=value]"
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity-mode > $OUT/a3_$i.log 2>&1 || exit 1
  env $2 timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity-mode > $OUT/b3_$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/acp_$i.log 2>&1 || exit 1
  env $2 timeout -k 10 200 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/bcp_$i.log 2>&1 || exit 1
done
for f in $OUT/a3_*.log $OUT/b3_*.log $OUT/acp_*.log $OUT/bcp_*.log; do
  echo "$(basename $f) $(tail -n 1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_roofline"]["stages"]; print(d["value"], d["ms_per_step"], "sparse_fwd", s["sparse_fwd"]["avg_ms"], "sparse_bwd", s["sparse_bwd"]["avg_ms"])')"
done
