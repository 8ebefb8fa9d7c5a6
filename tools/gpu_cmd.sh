mkdir -p gpurun_out/r01h
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_tail.py tests/test_gpu_anchor_head.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r01h/t.log 2>&1; echo "rc=$?"
tail -15 gpurun_out/r01h/t.log
