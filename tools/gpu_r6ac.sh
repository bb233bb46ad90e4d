# Round 6: refresh the PMC HBM traffic the bench lines quote, for the configs whose GEMMs changed this round
# (C4: fused LoRA down-projection; C5: second-segment spread refill) and C3 (attention barriers)
set -o pipefail
for M in sdxl-lora flux sdxl; do
  bash tools/gpu_pmc.sh r6_$M --model $M > gpurun_out/pmc_r6_$M.out 2>&1 || { tail -20 gpurun_out/pmc_r6_$M.out; exit 1; }
  echo "$M done"; tail -c 300 gpurun_out/pmc_r6_$M.json; echo
done
