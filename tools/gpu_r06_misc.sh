set -o pipefail
mkdir -p gpurun_out/r06misc
export TMPDIR=/tmp
RPC_PERT_ACT16=3 bash tools/gpu_pmc_traffic.sh r06misc_pmc_act16 "pert" > gpurun_out/r06misc/pmc_act16.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --model centerpoint --steps 10 --warmup 4 --no-parity-mode > gpurun_out/r06misc/bench_cp.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model strong --steps 30 --warmup 10 --no-parity-mode > gpurun_out/r06misc/bench_strong.log 2>&1 &&
tail -1 gpurun_out/r06misc/bench_cp.log | cut -c1-200 && tail -1 gpurun_out/r06misc/bench_strong.log | cut -c1-200 && head -12 gpurun_out/r06misc/pmc_act16.txt
