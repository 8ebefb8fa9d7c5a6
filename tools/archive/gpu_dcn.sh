#!/bin/bash
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/dcn_bench.py 0.0 > $OUT/dcn.log 2>&1 &&
timeout -k 10 120 python -u tools/dcn_bench.py 0.7 >> $OUT/dcn.log 2>&1 &&
cat $OUT/dcn.log &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex 'k_bwd' --output-format csv -d $OUT/pmc -o run -- python -u tools/dcn_bench.py 0.0 > $OUT/pmc.log 2>&1
RC=$?
F=$(find $OUT/pmc -name '*counter_collection.csv' | head -1)
[ -n "$F" ] && python - "$F" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    acc[r.get("Counter_Name")].append(float(r.get("Counter_Value", 0)))
for k, v in acc.items():
    print(f"{k}: mean per dispatch {sum(v)/len(v):.4g} (n={len(v)})")
PY
exit $RC
