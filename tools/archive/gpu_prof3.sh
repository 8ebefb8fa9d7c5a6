#!/bin/bash
# rocprofv3 kernel-trace of the KITTI 3-class bench step (hidden [64,128,64] perturber).
#   gpurun --timeout 600 -- bash tools/gpu_prof3.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-p3}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python -u bench.py --steps 12 --warmup 6 --no-cpu-baseline --classes 3 "$@" > $OUT/prof_bench.log 2>&1
RC=$?
KT=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
[ -n "$KT" ] && python tools/prof_summary.py $KT --steps 8 --top 70 > $OUT/step_kernels.txt 2>&1
[ -n "$KT" ] && gzip -c $KT > $OUT/kernel_trace.csv.gz
find $OUT/prof -name '*.csv' -size +4M -delete 2>/dev/null
find $OUT/prof -name '*.db' -delete 2>/dev/null
exit $RC
