#!/bin/bash
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
bash tools/gpu_cmd.sh $1 tests/test_gpu_dcn_head.py > /dev/null &&
timeout -k 10 120 python -u tools/dcn_bench.py 0.0 > $OUT/dcn.log 2>&1 &&
timeout -k 10 120 python -u tools/dcn_bench.py 0.7 >> $OUT/dcn.log 2>&1
RC=$?
tail -3 $OUT/pytest.log; cat $OUT/dcn.log
exit $RC
