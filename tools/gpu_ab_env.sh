#!/bin/bash
# short same-box bench A/B over environment settings: [REPS=n] tools/gpu_ab_env.sh TAG "ENV1" "ENV2" ...  (ENV "-" = defaults)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for rep in $(seq 1 ${REPS:-2}); do
  for e in "$@"; do
    i=$((i+1))
    envs=""; [ "$e" != "-" ] && envs="$e"
    env $envs timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-parity-mode --no-cpu-baseline \
      > $OUT/ab_${i}.log 2>&1 || exit $?
    python - "$OUT/ab_${i}.log" "$e" <<'PY'
import json, sys
ln = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(ln)
st = d.get("stage_roofline", {}).get("stages", {})
pr = d.get("perturber_roofline", {})
print(f"{sys.argv[2]:40s} {d['value']:8.1f} frames/s {d['ms_per_step']:.3f} ms  " +
      " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in st.items()) + "  " +
      " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in pr.items()))
PY
  done
done
