#!/bin/bash
# Per-kernel A/B of two library builds on the same box: rocprofv3 kernel stats of a short bench run
# with RPC_HIP_LIB=<base .so> (A) and the in-tree build (B), then a side-by-side table.
#   gpurun --timeout 900 -- bash tools/gpu_kernel_ab.sh <tag> <base.so> [filter-regex]
set -o pipefail
TAG=$1; BASE=$2; FILT=${3:-.}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$1 -o run -- \
    python -u bench.py --steps 10 --warmup 6 --no-cpu-baseline > $OUT/bench_$1.log 2>&1
}
RPC_HIP_LIB=$BASE run A && run B
RC=$?
python - "$OUT" "$FILT" <<'PY'
import csv, glob, re, sys, json
out, filt = sys.argv[1], sys.argv[2]
def stats(tag):
    f = glob.glob(f"{out}/prof_{tag}/**/*kernel_stats.csv", recursive=True)[0]
    return {r["Name"].split("(")[0]: (float(r["AverageNs"]) / 1e3, int(r["Calls"])) for r in csv.DictReader(open(f))}
a, b = stats("A"), stats("B")
for k in sorted(set(a) | set(b), key=lambda k: -(a.get(k, (0, 0))[0] * a.get(k, (0, 1))[1])):
    if not re.search(filt, k):
        continue
    x, y = a.get(k, (0, 0)), b.get(k, (0, 0))
    print(f"{x[0]:8.1f} {y[0]:8.1f} {y[0] - x[0]:+7.1f} us  x{y[1]:<4d} {k[:90]}")
for t in "AB":
    d = json.loads(open(f"{out}/bench_{t}.log").read().strip().splitlines()[-1])
    print(t, d["value"], d["ms_per_step"])
PY
exit $RC
