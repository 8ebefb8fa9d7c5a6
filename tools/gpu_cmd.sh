mkdir -p gpurun_out/r01j
timeout -k 10 200 python -u tools/host_profile.py --steps 20 > gpurun_out/r01j/host.txt 2>&1; echo "rc=$?"
