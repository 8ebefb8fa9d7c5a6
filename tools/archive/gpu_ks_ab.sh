set -o pipefail
OUT=gpurun_out/r05ks
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16_kernels.py tests/test_gpu_sparse_pipe.py tests/test_gpu_sparse_basicblock.py > $OUT/pytest.log 2>&1 && tail -n 1 $OUT/pytest.log &&
timeout -k 10 200 python -u tools/spwg_bench.py centerpoint fwd,dgrad > $OUT/a.log 2>&1 &&
RPC_HIP_LIB=$PWD/robustpointclouds_amd/_lib/librpc_hip_ab.so timeout -k 10 200 python -u tools/spwg_bench.py centerpoint fwd,dgrad > $OUT/b.log 2>&1
