#!/bin/bash
# same-box A/B of the pipelined S1 loops (knob 4: 0 = pipelined, 128 = former loop), x and y at the SECOND shapes
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
VARIANT=3 DBGS=0,128 SHAPES="6,100,88,256,256;6,200,176,128,128;6,100,88,128,256" timeout -k 10 200 python -u tools/conv_dbg_ab.py > $OUT/x.log 2>&1 && cat $OUT/x.log &&
VARIANT=4 DBGS=0,128 SHAPES="6,100,88,256,256;6,200,176,128,128;6,200,176,128,256" timeout -k 10 200 python -u tools/conv_dbg_ab.py > $OUT/y.log 2>&1 && cat $OUT/y.log
