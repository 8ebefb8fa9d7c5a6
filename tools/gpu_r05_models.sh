#!/bin/bash
# r05: step profile of the headline (3-class) bench, then the config-4 (CenterPoint) and config-5 (strong)
# bench lines with their own step profiles: tools/gpu_r05_models.sh <tag>
set -o pipefail
T=$1
bash tools/gpu_prof_model.sh ${T}_3class --steps 30 --warmup 10 &&
bash tools/gpu_prof_model.sh ${T}_cp --model centerpoint --steps 10 --warmup 4 &&
bash tools/gpu_prof_model.sh ${T}_strong --model strong --steps 20 --warmup 6
