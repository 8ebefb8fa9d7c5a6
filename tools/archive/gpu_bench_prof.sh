#!/bin/bash
# bench (headline + fp32 parity mode + CPU baseline) and a kernel-trace profile of the bf16 step
#   gpurun --timeout 900 -- bash tools/gpu_bench_prof.sh <tag>
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-300 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --steps 12 --warmup 6 --no-cpu-baseline --no-parity-mode > $OUT/prof_bench.log 2>&1 && echo "prof ok"
RC=$?
KT=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
[ -n "$KT" ] && python tools/prof_summary.py $KT --steps 8 --top 70 > $OUT/step_kernels.txt 2>&1
find $OUT/prof -name '*.csv' -size +4M -delete 2>/dev/null
find $OUT/prof -name '*.db' -delete 2>/dev/null
exit $RC
