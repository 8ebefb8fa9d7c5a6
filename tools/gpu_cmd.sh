O=gpurun_out/r01u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_pipeline.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; echo "rc=$?"; tail -25 $O/t.log
