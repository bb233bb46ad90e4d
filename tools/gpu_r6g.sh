# Round 6: C4 kernel trace with the fused LoRA down-projection (timeline + kernel stats) and the fused-form coverage.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu_profile.sh r6g sdxl-lora
