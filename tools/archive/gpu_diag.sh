#!/bin/bash
# Diagnostics in one call: host-issue gap of the 3-class step, then SQ / HBM counters for the
# kernels matching a regex.   gpurun -- bash tools/gpu_diag.sh <tag> <regex>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 200 python -u tools/host_gap.py --steps 20 --classes 3 > $OUT/host_gap.log 2>&1 &&
bash tools/gpu_pmc_step.sh $1 "$2"
