mkdir -p gpurun_out/r01g
timeout -k 10 300 python -u -m pytest tests/test_gpu_anchor_head.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r01g/head.log 2>&1; echo "head rc=$?"
tail -3 gpurun_out/r01g/head.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01g/prof -o run -- python -u bench.py --steps 8 --warmup 4 --no-cpu-baseline > gpurun_out/r01g/pb.log 2>&1
tail -1 gpurun_out/r01g/pb.log | cut -c1-200
python tools/prof_summary.py $(find gpurun_out/r01g/prof -name '*kernel_trace.csv') --steps 6 --top 80 > gpurun_out/r01g/sk.txt
grep -E "head|igemm<3>|wgrad<3>|wall" gpurun_out/r01g/sk.txt
find gpurun_out/r01g/prof -name '*.csv' -size +4M -delete
