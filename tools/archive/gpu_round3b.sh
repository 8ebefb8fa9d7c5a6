#!/bin/bash
# Round checkpoint (extended): full GPU suite, smoke, bench (bf16 headline + fp32 parity mode + Car + strong
# variant + CenterPoint), kernel-trace profile
#   gpurun --timeout 1200 -- bash tools/gpu_round3b.sh <tag>
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo "tests ok" && tail -1 $OUT/pytest_gpu.log &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $OUT/bench.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 8 --fp32 --no-cpu-baseline > $OUT/bench_fp32.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 8 --classes 1 --no-cpu-baseline > $OUT/bench_car.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 8 --model strong --no-cpu-baseline > $OUT/bench_strong.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --model centerpoint --no-cpu-baseline > $OUT/bench_centerpoint.log 2>&1 &&
echo "bench ok" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python -u bench.py --steps 12 --warmup 6 --no-cpu-baseline > $OUT/prof_bench.log 2>&1 && echo "prof ok"
RC=$?
for f in bench bench_fp32 bench_car bench_strong bench_centerpoint; do [ -f $OUT/$f.log ] && python -c "
import json; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))"; done
KT=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
[ -n "$KT" ] && python tools/prof_summary.py $KT --steps 8 --top 70 > $OUT/step_kernels.txt 2>&1
[ -n "$KT" ] && gzip -c $KT > $OUT/kernel_trace.csv.gz
find $OUT/prof -name '*.csv' -size +4M -delete 2>/dev/null
find $OUT/prof -name '*.db' -delete 2>/dev/null
exit $RC
