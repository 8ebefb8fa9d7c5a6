#!/bin/bash
# dense-engine tests, then bench.py with the fused BN-backward sums on / off (RPC_DENSE_BNFUSE), twice
#   gpurun --timeout 900 -- bash tools/gpu_bnfuse_ab.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense_bev.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do for f in 1 0; do
  RPC_DENSE_BNFUSE=$f timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench_f${f}_$rep.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('$OUT/bench_f${f}_$rep.log').read().strip().splitlines()[-1])
print('fuse=$f', d['value'], d['ms_per_step'], [(k['kernel'][-22:], k['avg_launch_ms'], k['launches']) for k in d.get('roofline_kernels', [])])"
done; done
