#!/bin/bash
# PMC pass over the conv microbench (one kernel variant): SQ occupancy / wait / MFMA / LDS counters.
set -o pipefail
OUT=gpurun_out/$1
VAR=${2:-0}
REGEX=${3:-k_conv3x3}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-include-regex "$REGEX" --output-format csv -d $OUT/pmc -o run -- python -u tools/conv_bench.py --variants $VAR --rounds 1 --iters 2 > $OUT/pmc.log 2>&1
RC=$?
F=$(find $OUT/pmc -name '*counter_collection.csv' | head -1)
[ -n "$F" ] && python - "$F" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    acc[(r.get("Kernel_Name")[:40], r.get("Grid_Size"))][r.get("Counter_Name")].append(float(r.get("Counter_Value", 0)))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c}: {sum(v)/len(v):.4g} (n={len(v)})")
    wc = sum(d["SQ_WAVE_CYCLES"]) or 1
    print("   wait_any/wave %.3f  wait_inst/wave %.3f  active/wave %.3f  lds_conflict/lds_active %.3f" % (
        sum(d["SQ_WAIT_ANY"]) / wc, sum(d["SQ_WAIT_INST_ANY"]) / wc, sum(d["SQ_ACTIVE_INST_ANY"]) / wc,
        sum(d["SQ_LDS_BANK_CONFLICT"]) / max(sum(d["SQ_LDS_IDX_ACTIVE"]), 1)))
PY
find $OUT/pmc -name '*.csv' -size +4M -delete 2>/dev/null
exit $RC
