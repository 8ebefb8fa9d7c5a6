#!/bin/bash
# pytest subset, then a short KITTI bench (no cpu baseline)
set -o pipefail
T=$1; shift
bash tools/gpu_cmd.sh $T "$@" &&
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/$T/bench.log 2>&1
RC=$?
tail -1 gpurun_out/$T/bench.log | cut -c1-200
python - <<'PY' "gpurun_out/$T/bench.log"
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d.get("roofline", {})
    print("roofline", r.get("achieved"), r.get("frac"), r.get("avg_launch_ms"))
except Exception as e:
    print("no bench json", e)
PY
exit $RC
