#!/bin/bash
# Per-kernel perturber durations at two voxel counts (tools/pert_bench.py under rocprofv3 kernel trace):
#   tools/gpu_pert_prof.sh <tag>   -> gpurun_out/<tag>/v<V>/run_results.db
set -o pipefail
OUT=$PWD/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for V in 10000 80000; do
  timeout -k 10 150 rocprofv3 --kernel-trace -d $OUT/v$V -o run -- python3 $GRAFT_REPO_ROOT/tools/pert_bench.py $V > $OUT/v$V.log 2>&1 || exit 1
done
