# Refresh the per-config HBM traffic JSONs bench.py quotes (profiles/pmc_traffic_*.json): two PMC passes per model.
set -o pipefail
for M in sd15 sdxl-lora flux sdxl; do
  bash tools/gpu_pmc.sh r5_$M --model $M > gpurun_out/pmc_r5_$M.out 2>&1 || { tail -20 gpurun_out/pmc_r5_$M.out; exit 1; }
  echo "$M done"; tail -c 600 gpurun_out/pmc_r5_$M.json; echo
done
