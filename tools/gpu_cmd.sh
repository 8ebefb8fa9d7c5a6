O=gpurun_out/r01t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_strong_variant.py tests/test_gpu_dense_bev.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; echo "rc=$?"; tail -4 $O/t.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 8 --no-cpu-baseline > $O/b1.log 2>&1 && tail -1 $O/b1.log | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline > $O/pb1.log 2>&1
python tools/prof_summary.py $(find $O/prof1 -name '*kernel_trace.csv') --steps 8 --top 40 > $O/sk1.txt
grep -E "wall|bn" $O/sk1.txt
find $O/prof1 -name '*.csv' -size +4M -delete
