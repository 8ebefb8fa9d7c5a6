#!/bin/bash
# pytest subset, then the CenterPoint bench + profile
set -o pipefail
T=$1; shift
bash tools/gpu_cmd.sh $T "$@" && bash tools/gpu_cp.sh $T
