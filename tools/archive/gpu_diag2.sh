#!/bin/bash
# host phases + a kernel-trace profile of the bench (no tests)
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/host_phases.py --steps 20 > $OUT/host_phases.log 2>&1 && cat $OUT/host_phases.log &&
bash tools/gpu_round.sh $TAG profonly
