#!/bin/bash
# kernel-trace profile of the default bench: per-kernel step table + one step's timeline (start, duration, stream)
#   tools/gpu_prof_timeline.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py "$@" --steps 8 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/prof_bench.log 2>&1 || exit $?
KT=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python tools/prof_summary.py $KT --steps 4 --top 80 > $OUT/step_kernels.txt 2>&1
python tools/trace_timeline.py $KT --step 6 > $OUT/timeline.txt 2>&1
cp $(find $OUT/prof -name '*kernel_stats.csv' | head -1) $OUT/kernel_stats.csv 2>/dev/null
find $OUT/prof -name '*.csv' -size +4M -delete 2>/dev/null
find $OUT/prof -name '*.db' -delete 2>/dev/null
echo "prof ok"
