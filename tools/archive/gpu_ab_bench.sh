#!/bin/bash
# bench A/B over env switches: tools/gpu_ab_bench.sh <tag> "<ENV=..>" "<ENV=..>" ...
# ("default" = no switch); one line per variant: ms/step, frames/s, sparse / perturber stage times
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then E=""; else E="$v"; fi
  env $E timeout -k 10 200 python -u bench.py $BENCH_ARGS --steps 30 --warmup 8 --no-cpu-baseline --no-parity-mode \
    > "$OUT/ab_${v// /_}.log" 2>&1 || exit $?
  python - "$OUT/ab_${v// /_}.log" "$v" <<'PY' | tee -a $OUT/ab.txt
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
r = json.loads(line)
st = {k: v["avg_ms"] for k, v in r.get("stage_roofline", {}).get("stages", {}).items()}
print(f'{sys.argv[2]:40s} {r["ms_per_step"]:.3f} ms/step {r["value"]:.1f} fps  stages {st}')
PY
done
