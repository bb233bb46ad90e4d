set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/host_bound_probe.py --steps 8 --rounds 2 --lead-ms 10 30 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4f_probe.txt
