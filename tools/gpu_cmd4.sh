#!/bin/bash
set -o pipefail
T=$1; shift
timeout -k 10 200 python -u tools/bnfin_bench.py > /tmp/bnfin.log 2>&1; grep nblk /tmp/bnfin.log
bash tools/gpu_cmd3.sh $T "$@"
