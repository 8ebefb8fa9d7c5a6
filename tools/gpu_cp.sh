#!/bin/bash
# CenterPoint bench + kernel profile in one call
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline > $OUT/bench_cp.log 2>&1 &&
tail -1 $OUT/bench_cp.log | cut -c1-600 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python -u bench.py --model centerpoint --steps 6 --warmup 3 --no-cpu-baseline > $OUT/prof_bench.log 2>&1
RC=$?
KT=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
[ -n "$KT" ] && python tools/prof_summary.py $KT --steps 6 --top 45 > $OUT/step_kernels.txt 2>&1
find $OUT/prof -name '*.csv' -size +4M -delete 2>/dev/null
find $OUT/prof -name '*.db' -delete 2>/dev/null
exit $RC
