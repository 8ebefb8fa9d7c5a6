O=gpurun_out/r01q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_perturber.py tests/test_adversarial_voxelnet.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; echo "rc=$?"; tail -2 $O/t.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 8 --classes 3 --no-cpu-baseline > $O/b3.log 2>&1 && tail -1 $O/b3.log | cut -c1-200
timeout -k 10 200 python -u bench.py --steps 20 --warmup 8 --no-cpu-baseline > $O/b1.log 2>&1 && tail -1 $O/b1.log | cut -c1-200
for C in 3 1; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$C -o run -- python -u bench.py --steps 10 --warmup 5 --classes $C --no-cpu-baseline > $O/pb$C.log 2>&1
python tools/prof_summary.py $(find $O/prof$C -name '*kernel_trace.csv') --steps 8 --top 40 > $O/sk$C.txt
grep -E "wall|pert" $O/sk$C.txt
find $O/prof$C -name '*.csv' -size +4M -delete
done
