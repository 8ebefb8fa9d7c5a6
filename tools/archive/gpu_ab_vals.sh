#!/bin/bash
# A/B/.. of one environment variable over several values on the same box: bench.py (3-class), the values
# interleaved, REPS rounds (default 2); optional pytest file run first with the first value
#   gpurun --timeout 900 -- bash tools/gpu_ab_vals.sh <tag> <VAR> "<v1> <v2> ..." [pytest-file] [reps]
set -o pipefail
OUT=gpurun_out/$1
VAR=$2
VALS=$3
TESTF=$4
REPS=${5:-2}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTF" ]; then
  timeout -k 10 300 python -u -m pytest $TESTF -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for rep in $(seq 1 $REPS); do for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench_${v}_$rep.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('$OUT/bench_${v}_$rep.log').read().strip().splitlines()[-1]); st=d.get('stage_roofline',{}).get('stages',{})
print('$VAR=$v', d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in st.items()})"
done; done
