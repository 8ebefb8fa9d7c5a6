#!/bin/bash
# whole-step A/B of library builds (RPC_HIP_LIB=<.so> per arm, "-" = the in-tree build): bench.py 3-class,
# frames/s and the HBM stage timings (voxelize / perturber / sparse), interleaved twice
#   gpurun --timeout 900 -- bash tools/gpu_lib_ab.sh <tag> <so|-> [<so|-> ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in "$@"; do
    name=$(basename $lib .so); [ "$lib" = "-" ] && name=intree
    if [ "$lib" = "-" ]; then
      timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench_${name}_$rep.log 2>&1 || exit 1
    else
      RPC_HIP_LIB=$(realpath $lib) timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > $OUT/bench_${name}_$rep.log 2>&1 || exit 1
    fi
    python -c "
import json; d=json.loads(open('$OUT/bench_${name}_$rep.log').read().strip().splitlines()[-1])
st=d.get('stage_roofline',{}).get('stages',{})
print('$name', $rep, d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in st.items()})"
  done
done
