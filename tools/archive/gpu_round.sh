#!/bin/bash
# One gpurun call: GPU tests, bench, rocprof kernel-trace stats. Each GPU step has its own
# time limit; steps are chained with && so a failure ends the call.
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh <tag> [tests|notests]
set -o pipefail
TAG=${1:-x}
MODE=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step_tests() {
  [ "$MODE" != "tests" ] && [ "$MODE" != "all" ] && return 0
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1
}
step_bench() {
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $OUT/bench.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 8 --classes 1 --no-cpu-baseline > $OUT/bench_car.log 2>&1
}
step_prof() {
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --steps 12 --warmup 6 --no-cpu-baseline > $OUT/prof_bench.log 2>&1
}
step_pmc() {
  [ "$MODE" != "pmc" ] && [ "$MODE" != "all" ] && return 0
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --kernel-include-regex 'k_conv3x3|k_wgrad|k_gemm_bf16|k_bnbwd' \
      --output-format csv -d $OUT/pmc_$C -o run -- \
      python -u bench.py --steps 4 --warmup 3 --no-cpu-baseline > $OUT/pmc_$C.log 2>&1 || return 1
  done
  python tools/pmc_traffic.py $(find $OUT/pmc_FETCH_SIZE -name '*counter_collection.csv') \
    $(find $OUT/pmc_WRITE_SIZE -name '*counter_collection.csv') $OUT/pmc_traffic.json 40 > $OUT/pmc_traffic.txt 2>&1
}
step_tests && echo "tests ok" && { [ "$MODE" = "profonly" ] || { step_bench && echo "bench ok" && tail -1 $OUT/bench.log | cut -c1-400; tail -1 $OUT/bench_car.log | cut -c1-300; }; } && step_prof && echo "prof ok" && step_pmc && echo "pmc ok"
RC=$?
KT=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
[ -n "$KT" ] && python tools/prof_summary.py $KT --steps 8 --top 60 > $OUT/step_kernels.txt 2>&1
[ -n "$KT" ] && gzip -c $KT > $OUT/kernel_trace.csv.gz
find $OUT/prof -name '*.csv' -size +4M -delete 2>/dev/null
find $OUT/prof -name '*.json' -size +4M -delete 2>/dev/null
find $OUT/prof -name '*.db' -delete 2>/dev/null
ls -laR $OUT > $OUT/ls.txt
exit $RC
