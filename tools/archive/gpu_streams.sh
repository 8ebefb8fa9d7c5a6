#!/bin/bash
# kernel trace of the bench step -> per-stream busy, GPU idle gaps (tools/step_streams.py): tools/gpu_streams.sh <tag> [bench args]
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py "$@" --steps 8 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/prof_bench.log 2>&1 && echo "prof ok"
RC=$?
KT=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
[ -n "$KT" ] && python tools/step_streams.py $KT --steps 4 --top 25 > $OUT/streams.txt 2>&1 && \
  python tools/prof_summary.py $KT --steps 4 --top 60 > $OUT/step_kernels.txt 2>&1 && gzip -f $KT
find $OUT/prof -name '*.db' -delete 2>/dev/null
exit $RC
