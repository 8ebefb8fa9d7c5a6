#!/bin/bash
# BatchNorm finalize A/B (in-tree default a vs RPC_BN_FIN_WIDE=0 b): finalize / sparse / CenterPoint GPU tests, then
# the CenterPoint and 3-class bench lines alternating: tools/gpu_bnfin_ab.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bn_finalize.py tests/test_gpu_sparse_pipe.py tests/test_gpu_sparse_encoder.py tests/test_gpu_centerpoint.py > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/acp_$i.log 2>&1 || exit 1
  RPC_BN_FIN_WIDE=0 timeout -k 10 200 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/bcp_$i.log 2>&1 || exit 1
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity-mode > $OUT/a3_$i.log 2>&1 || exit 1
  RPC_BN_FIN_WIDE=0 timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity-mode > $OUT/b3_$i.log 2>&1 || exit 1
done
tail -n 1 $OUT/pytest.log
for f in $OUT/acp_*.log $OUT/bcp_*.log $OUT/a3_*.log $OUT/b3_*.log; do
  echo "$(basename $f) $(tail -n 1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["stage_roofline"]["stages"]; print(d["value"], d["ms_per_step"], "sparse_fwd", s["sparse_fwd"]["avg_ms"], "sparse_bwd", s["sparse_bwd"]["avg_ms"])')"
done
