#!/bin/bash
# selected GPU tests, then a rocprof kernel trace of the 3-class bench step
#   gpurun --timeout 900 -- bash tools/gpu_tests_prof.sh <tag> <test files...>
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && echo tests ok &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u bench.py --steps 12 --warmup 6 --no-cpu-baseline > $OUT/prof_bench.log 2>&1
RC=$?
KT=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
[ -n "$KT" ] && python tools/prof_summary.py $KT --steps 8 --top 200 > $OUT/step_kernels.txt 2>&1
[ -n "$KT" ] && gzip -c $KT > $OUT/kernel_trace.csv.gz
find $OUT/prof -name '*.csv' -size +1M -delete 2>/dev/null
find $OUT/prof -name '*.db' -delete 2>/dev/null
tail -3 $OUT/pytest.log
exit $RC
