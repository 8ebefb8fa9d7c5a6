#!/bin/bash
# bench + kernel-trace profile of one model: tools/gpu_prof_model.sh <tag> <bench args...>
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py "$@" > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-400 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py "$@" --steps 8 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/prof_bench.log 2>&1 && echo "prof ok"
RC=$?
KT=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
[ -n "$KT" ] && python tools/prof_summary.py $KT --steps 4 --top 60 > $OUT/step_kernels.txt 2>&1
find $OUT/prof -name '*.csv' -size +4M -delete 2>/dev/null
find $OUT/prof -name '*.db' -delete 2>/dev/null
exit $RC
