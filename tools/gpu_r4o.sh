# PMC passes over the dual-image attention kernels at SDXL level 1 / level 2
set -o pipefail
bash tools/gpu_attn_pmc.sh r4o_l1 4 4096 4096 10 64 > gpurun_out/r4o_l1.txt 2>&1 || { cat gpurun_out/r4o_l1.txt; exit 1; }
bash tools/gpu_attn_pmc.sh r4o_l2 4 1024 1024 20 64 > gpurun_out/r4o_l2.txt 2>&1 || { cat gpurun_out/r4o_l2.txt; exit 1; }
cat gpurun_out/r4o_l1.txt gpurun_out/r4o_l2.txt
