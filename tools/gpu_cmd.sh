O=gpurun_out/r01v
mkdir -p $O
timeout -k 10 200 python -u bench.py --steps 20 --warmup 8 --classes 3 --model strong --no-cpu-baseline > $O/bs.log 2>&1; echo rc=$?; tail -1 $O/bs.log | cut -c1-330
timeout -k 10 200 python -u bench.py --steps 20 --warmup 8 --classes 3 --no-cpu-baseline > $O/b3.log 2>&1 && tail -1 $O/b3.log | cut -c1-200
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo smoke rc=$?; tail -1 $O/smoke.log | cut -c1-300
