# Round 6: host issue vs GPU time per step at HEAD, C3 and C4 (tools/host_overhead.py)
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_overhead.py > gpurun_out/r6_host_overhead_sdxl.txt 2>&1 || { tail -20 gpurun_out/r6_host_overhead_sdxl.txt; exit 1; }
HO_LORA=32 timeout -k 10 300 python -u tools/host_overhead.py > gpurun_out/r6_host_overhead_sdxl-lora.txt 2>&1 || { tail -20 gpurun_out/r6_host_overhead_sdxl-lora.txt; exit 1; }
grep step gpurun_out/r6_host_overhead_sdxl.txt | head -5; grep step gpurun_out/r6_host_overhead_sdxl-lora.txt | head -5
