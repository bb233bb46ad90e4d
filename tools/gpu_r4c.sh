set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/attn_determinism.py --reps 20 2>&1 | grep -v amdgpu.ids
OTAMD_ATTN_XCD=0 timeout -k 10 200 python -u tools/attn_determinism.py --reps 20 2>&1 | grep -v amdgpu.ids
OTAMD_ATTN_CROSS_OFF=1 timeout -k 10 200 python -u tools/attn_determinism.py --reps 20 2>&1 | grep -v amdgpu.ids
