#!/bin/bash
# PMC passes over the sparse bf16 GEMM kernels (two passes: issue/wait mix, then memory)
set -o pipefail
OUT=gpurun_out/$1
REGEX=${2:-k_gemm_bf16}
mkdir -p $OUT
export TMPDIR=/tmp
summ() {
python - "$1" <<'PY'
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
}
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "$REGEX" --output-format csv -d $OUT/p1 -o run -- python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/p1.log 2>&1 &&
summ $(find $OUT/p1 -name '*counter_collection.csv' | head -1) > $OUT/p1.txt &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$REGEX" --output-format csv -d $OUT/p2 -o run -- python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/p2.log 2>&1 &&
summ $(find $OUT/p2 -name '*counter_collection.csv' | head -1) > $OUT/p2.txt
RC=$?
find $OUT -name '*.csv' -size +4M -delete 2>/dev/null
cat $OUT/p1.txt $OUT/p2.txt
exit $RC
