#!/bin/bash
# kernel-trace profile of the default bench under an env switch: tools/gpu_prof_env.sh <tag> "<ENV=..>"
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export $2
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --steps 12 --warmup 6 --no-cpu-baseline --no-parity-mode > $OUT/prof_bench.log 2>&1 && echo "prof ok"
RC=$?
KT=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
[ -n "$KT" ] && python tools/prof_summary.py $KT --steps 8 --top 70 > $OUT/step_kernels.txt 2>&1
find $OUT/prof -name '*.csv' -size +4M -delete 2>/dev/null
find $OUT/prof -name '*.db' -delete 2>/dev/null
exit $RC
