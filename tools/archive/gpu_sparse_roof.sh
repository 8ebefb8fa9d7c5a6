#!/bin/bash
set -o pipefail
for k in fwd,64,64 dgrad,64,64 wgrad,64,64 fwd,32,32 wgrad,32,32; do
  timeout -k 10 200 python -u bench.py --steps 8 --warmup 4 --no-cpu-baseline --roofline-kernel $k 2>/dev/null | tail -1 | python -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('$k', r['kernel'][:60], 'TF/s', r['achieved'], 'frac', r['frac'], 'ms', r['avg_launch_ms'], 'GF', round(r['flops_per_launch']/1e9,2))" || exit 1
done
