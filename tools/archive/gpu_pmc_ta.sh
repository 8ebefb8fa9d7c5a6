#!/bin/bash
# one PMC pass with the texture-addresser busy counter next to the SQ issue/wait mix
set -o pipefail
OUT=gpurun_out/$1
REGEX=${2:-k_wgrad}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU TA_TA_BUSY_sum GRBM_GUI_ACTIVE --kernel-include-regex "$REGEX" --output-format csv -d $OUT/pmc -o run -- python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/pmc.log 2>&1
RC=$?
F=$(find $OUT/pmc -name '*counter_collection.csv' | head -1)
[ -n "$F" ] && python - "$F" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    acc[r.get("Kernel_Name")[:60]][r.get("Counter_Name")].append(float(r.get("Counter_Value", 0)))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c}: {sum(v)/len(v):.4g} (n={len(v)})")
PY
find $OUT -name '*.csv' -size +4M -delete 2>/dev/null
tail -3 $OUT/pmc.log
exit $RC
