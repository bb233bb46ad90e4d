# Round 6: C4 determinism bisection -- 24 runs per variant
set -o pipefail
bash tools/gpu_r6v.sh r6x_b48 24 OTAMD_NORM_BUCKET_MB=48 && \
bash tools/gpu_r6v.sh r6x_nodefer 24 OTAMD_DEFER_REDUCE=0 && \
bash tools/gpu_r6v.sh r6x_nolndefer 24 OTAMD_LN_DEFER=0
