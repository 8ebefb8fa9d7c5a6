#!/bin/bash
# HBM traffic per launch of every kernel of a short bench.py run: two rocprofv3 --pmc passes (FETCH_SIZE,
# WRITE_SIZE; never combined with tracing), summarised by tools/pmc_traffic.py into <tag>/pmc_traffic.json
#   gpurun -- bash tools/gpu_pmc_traffic.sh <tag> [kernel regex]     (BENCH_ARGS="--model centerpoint" for config 4)
set -o pipefail
OUT=gpurun_out/$1
REGEX=${2:-.}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$REGEX" --output-format csv -d $OUT/pmc_f -o run -- python -u bench.py $BENCH_ARGS --steps 3 --warmup 2 --no-cpu-baseline --no-parity-mode > $OUT/pmc_f.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$REGEX" --output-format csv -d $OUT/pmc_w -o run -- python -u bench.py $BENCH_ARGS --steps 3 --warmup 2 --no-cpu-baseline --no-parity-mode > $OUT/pmc_w.log 2>&1
RC=$?
F=$(find $OUT/pmc_f -name '*counter_collection.csv' | head -1)
W=$(find $OUT/pmc_w -name '*counter_collection.csv' | head -1)
[ -n "$F" ] && [ -n "$W" ] && python tools/pmc_traffic.py "$F" "$W" $OUT/pmc_traffic.json 100000 > $OUT/pmc_traffic.txt 2>&1 && head -30 $OUT/pmc_traffic.txt
find $OUT -name '*.csv' -size +4M -delete 2>/dev/null
exit $RC
