set -o pipefail
OUT=gpurun_out/r05n32
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv_bench.py --knob 5 --variants 1,2 --shapes "4,128,128,64,64;4,128,128,320,64;4,128,128,64,320;4,64,64,64,256;4,64,64,256,256" > $OUT/conv.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dense_bev.py tests/test_gpu_dcn_head.py tests/test_gpu_center_head.py tests/test_gpu_centerpoint.py > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/acp_$i.log 2>&1 || exit 1
  RPC_DENSE_S1N32=1 timeout -k 10 200 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-cpu-baseline --no-parity-mode > $OUT/bcp_$i.log 2>&1 || exit 1
done
for f in $OUT/acp_*.log $OUT/bcp_*.log; do
  echo "$(basename $f) $(tail -n 1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
