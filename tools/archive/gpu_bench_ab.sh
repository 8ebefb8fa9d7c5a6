#!/bin/bash
# bench.py with the dense HIP graphs on and off, plus the host-gap check (3-class)
#   gpurun --timeout 900 -- bash tools/gpu_bench_ab.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $OUT/bench_graphs.log 2>&1 &&
RPC_DENSE_GRAPHS=0 timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench_eager.log 2>&1 &&
timeout -k 10 200 python -u tools/host_gap.py --steps 20 --classes 3 > $OUT/host_gap.log 2>&1
RC=$?
for f in bench_graphs bench_eager; do python -c "
import json,sys; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_launch_ms'))"; done
tail -2 $OUT/host_gap.log
exit $RC
