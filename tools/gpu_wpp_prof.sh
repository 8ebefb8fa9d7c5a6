set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06wpp_prof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/a -o run -- python -u bench.py --model centerpoint --steps 4 --warmup 2 --no-cpu-baseline --no-parity-mode > $OUT/a.log 2>&1 &&
RPC_HIP_LIB=$PWD/robustpointclouds_amd/_lib/librpc_hip_ab.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/b -o run -- python -u bench.py --model centerpoint --steps 4 --warmup 2 --no-cpu-baseline --no-parity-mode > $OUT/b.log 2>&1 &&
for v in a b; do f=$(find $OUT/$v -name '*kernel_stats.csv' | head -1); echo "== $v"; grep -E "k_wgrad_pp|k_wgrad_reduce|pert::k_bwd" $f | cut -d, -f1-6; done
find $OUT -name '*.csv' -size +2M -delete 2>/dev/null; find $OUT -name '*.db' -delete 2>/dev/null
