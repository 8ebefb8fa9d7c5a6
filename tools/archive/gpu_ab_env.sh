#!/bin/bash
# A/B of one environment toggle on the same box: bench.py (3-class) with VAR=1 then VAR=0, twice each
#   gpurun --timeout 900 -- bash tools/gpu_ab_env.sh <tag> <VAR>
set -o pipefail
OUT=gpurun_out/$1
VAR=$2
mkdir -p $OUT
export TMPDIR=/tmp
run() { env $VAR=$2 timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench_$1.log 2>&1; }
run on1 1 && run off1 0 && run on2 1 && run off2 0
RC=$?
for f in on1 off1 on2 off2; do python -c "
import json; d=json.loads(open('$OUT/bench_$f.log').read().strip().splitlines()[-1]); st=d.get('stage_roofline',{}).get('stages',{})
print('$f', d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in st.items()})"; done
exit $RC
