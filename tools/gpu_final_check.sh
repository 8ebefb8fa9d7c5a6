#!/bin/bash
# final tree check: full GPU suite, smoke, one 3-class bench
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && tail -1 $OUT/pytest_gpu.log &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | cut -c1-160
