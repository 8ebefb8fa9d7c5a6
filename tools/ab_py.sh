#!/bin/bash
# Same-box A/B of one Python module of the package: A = the tree, B = gpurun_ab/<module>_old.py (e.g.
# git show HEAD~:robustpointclouds_amd/<module>.py > gpurun_ab/<module>_old.py) swapped in; alternating A B A B:
#   tools/ab_py.sh <tag> <model> <module> [steps]
set -o pipefail
OUT=gpurun_out/$1; M=$2; F=$3; S=${4:-30}
mkdir -p $OUT; export TMPDIR=/tmp
cp robustpointclouds_amd/$F.py /tmp/new_$F.py
for i in 1 2; do
  cp /tmp/new_$F.py robustpointclouds_amd/$F.py
  timeout -k 10 300 python -u bench.py --model $M --steps $S --warmup 6 --no-cpu-baseline --no-parity-mode > $OUT/a_$i.log 2>&1 || exit 1
  cp gpurun_ab/${F}_old.py robustpointclouds_amd/$F.py
  timeout -k 10 300 python -u bench.py --model $M --steps $S --warmup 6 --no-cpu-baseline --no-parity-mode > $OUT/b_$i.log 2>&1 || exit 1
done
cp /tmp/new_$F.py robustpointclouds_amd/$F.py
for f in $OUT/a_*.log $OUT/b_*.log; do
  echo "$(basename $f) $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
