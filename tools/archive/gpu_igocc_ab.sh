set -o pipefail
OUT=gpurun_out/r05io
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/igemm_bench.py --knob 6 --variants 4,3 --only P1,U2,G2 > $OUT/igemm.txt 2>&1 || exit 1
RPC_DENSE_IGOCC=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dense_bev.py > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity-mode > $OUT/a3_$i.log 2>&1 || exit 1
  RPC_DENSE_IGOCC=3 timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-parity-mode > $OUT/b3_$i.log 2>&1 || exit 1
done
tail -n 1 $OUT/pytest.log
for f in $OUT/a3_*.log $OUT/b3_*.log; do echo "$(basename $f) $(tail -n 1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
