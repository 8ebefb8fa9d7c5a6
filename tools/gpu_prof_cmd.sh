#!/bin/bash
# kernel-trace stats of one python command: tools/gpu_prof_cmd.sh TAG script.py [args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u "$@" > $OUT/run.log 2>&1 || exit $?
cp $(find $OUT/prof -name '*kernel_stats.csv' | head -1) $OUT/kernel_stats.csv
find $OUT/prof -name '*.csv' -size +4M -delete 2>/dev/null
find $OUT/prof -name '*.db' -delete 2>/dev/null
cut -d, -f1-8 $OUT/kernel_stats.csv | head -30
