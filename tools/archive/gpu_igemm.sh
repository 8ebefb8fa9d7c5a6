#!/bin/bash
# dense implicit-GEMM microbench (S2/D2/P1/U2/G2 at the step's shapes) + PMC passes on it
#   gpurun --timeout 600 -- bash tools/gpu_igemm.sh <tag> [variants] [pmc]
set -o pipefail
OUT=gpurun_out/$1
VAR=${2:-0}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/igemm_bench.py --variants $VAR > $OUT/igemm.log 2>&1 || exit 1
cat $OUT/igemm.log
[ "$3" = "pmc" ] || exit 0
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'k_igemm' --output-format csv -d $OUT/pmc_$N -o run -- \
    python -u tools/igemm_bench.py --variants $VAR --rounds 1 --iters 2 > $OUT/pmc_$N.log 2>&1 || exit 1
done
python - $OUT <<'PY'
import csv, sys, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        key = r["Kernel_Name"].split("(")[0][-24:] + " grid=" + r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    print(k, " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items())))
PY
find $OUT -name '*.csv' -size +4M -delete 2>/dev/null
exit 0
