#!/bin/bash
# PMC pass over a short bench.py run for the kernels matching a regex: SQ occupancy / wait / MFMA /
# LDS counters, then (second pass) HBM bytes.   gpurun -- bash tools/gpu_pmc_step.sh <tag> <regex>
set -o pipefail
OUT=gpurun_out/$1
REGEX=$2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-include-regex "$REGEX" --output-format csv -d $OUT/pmc -o run -- python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/pmc.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$REGEX" --output-format csv -d $OUT/pmc_f -o run -- python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/pmc_f.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$REGEX" --output-format csv -d $OUT/pmc_w -o run -- python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/pmc_w.log 2>&1
RC=$?
python - $(find $OUT/pmc $OUT/pmc_f $OUT/pmc_w -name '*counter_collection.csv') <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        acc[r.get("Kernel_Name")[:60]][r.get("Counter_Name")].append(float(r.get("Counter_Value", 0)))
for k, d in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in d.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1) or 1
    print(k)
    print("   wait_any %.3f wait_inst %.3f active %.3f  mfma_busy %.4g busy %.4g  lds_conf %.3f  fetch(x2) %.1f MB write %.1f MB" % (
        m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc, m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0), m.get("SQ_BUSY_CYCLES", 0),
        m.get("SQ_LDS_BANK_CONFLICT", 0) / max(m.get("SQ_LDS_IDX_ACTIVE", 1), 1),
        2 * m.get("FETCH_SIZE", 0) / 1e3, m.get("WRITE_SIZE", 0) / 1e3))
PY
find $OUT -name '*.csv' -size +4M -delete 2>/dev/null
exit $RC
