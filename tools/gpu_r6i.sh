# Round 6: kernel traces of C5 (FLUX LoRA) and C2 (SD 1.5) at HEAD.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu_profile.sh r6i flux && bash tools/gpu_profile.sh r6i sd15
