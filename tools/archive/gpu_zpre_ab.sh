set -o pipefail
mkdir -p gpurun_out/r03_zpre
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense_bev.py -x -q --timeout 120 --timeout-method thread -k "fused_bn or wide_tile or config_shape" > gpurun_out/r03_zpre/pytest.log 2>&1 && tail -1 gpurun_out/r03_zpre/pytest.log &&
bash tools/gpu_lib_ab.sh r03_zpre ablib/base.so -
