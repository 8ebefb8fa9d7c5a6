#!/bin/bash
# whole-step A/B of the dense S1 kernel choice and the fused BatchNorm-backward sums (3-class bench)
#   gpurun --timeout 900 -- bash tools/gpu_bench_s1ab.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
for arm in "auto::" "x_only:RPC_DENSE_S1=3:" "x_nofuse:RPC_DENSE_S1=3:RPC_DENSE_BNFUSE=0" "auto_nofuse::RPC_DENSE_BNFUSE=0" "auto2::"; do
  name=${arm%%:*}; rest=${arm#*:}; e1=${rest%%:*}; e2=${rest#*:}
  env $e1 $e2 timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench_$name.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('$OUT/bench_$name.log').read().strip().splitlines()[-1])
print('$name', d['value'], d['ms_per_step'], [(k['kernel'][-16:], k['avg_launch_ms'], k['frac']) for k in d.get('roofline_kernels', [])])"
done
