#!/bin/bash
# L2 hit rate (TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)) per kernel of a short bench run, one --pmc pass:
#   tools/gpu_pmc_l2.sh <tag> [kernel regex]
set -o pipefail
OUT=gpurun_out/$1
REGEX=${2:-.}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$REGEX" --output-format csv -d $OUT/l2 -o run -- python -u bench.py $BENCH_ARGS --steps 3 --warmup 2 --no-cpu-baseline --no-parity-mode > $OUT/l2.log 2>&1
RC=$?
F=$(find $OUT/l2 -name '*counter_collection.csv' | head -1)
[ -n "$F" ] && python - "$F" > $OUT/l2.txt <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0][:70]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in sorted(acc.items(), key=lambda kv: -(kv[1].get("TCC_HIT_sum", 0) + kv[1].get("TCC_MISS_sum", 0))):
    h, m = d.get("TCC_HIT_sum", 0.0), d.get("TCC_MISS_sum", 0.0)
    if h + m > 0:
        print(f"{h / (h + m):6.3f} hit  {(h + m) / max(n[(k, 'TCC_HIT_sum')], 1):12.0f} req/launch  {k}")
PY
find $OUT -name '*.csv' -size +4M -delete 2>/dev/null
head -40 $OUT/l2.txt
exit $RC
