#!/bin/bash
# dense-engine GPU tests, S1 variants x (3) / y (4) at the SECOND shapes, then the 3-class bench twice
#   gpurun --timeout 900 -- bash tools/gpu_pipe_check.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense_bev.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && tail -2 $OUT/pytest.log &&
timeout -k 10 200 python -u tools/conv_bench.py --variants 3,4 > $OUT/conv_bench.log 2>&1 && cat $OUT/conv_bench.log &&
timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench1.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench2.log 2>&1 &&
for f in bench1 bench2; do python -c "
import json; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], [(k['kernel'][-22:], k['avg_launch_ms'], k['launches']) for k in d.get('roofline_kernels', [])])"; done
