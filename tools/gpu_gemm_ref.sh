# The engine's planned GEMM vs torch.matmul (hipBLASLt) on the SDXL step's dominant shapes, same random
# operands, median of 50 launches each (tools/gemm_one.py --torch).  usage: bash tools/gpu_gemm_ref.sh <tag>
set -o pipefail
TAG=$1
mkdir -p gpurun_out
OUT=gpurun_out/gemm_ref_${TAG}.jsonl
: > $OUT
while read -r OP M N K; do
  timeout -k 10 120 python3 -u tools/gemm_one.py $OP $M $N $K --torch --reps 50 >> $OUT || { echo "gemm_one $OP $M $N $K failed"; exit 1; }
done <<'EOF'
fwd 4096 4096 4096
fwd 8192 8192 8192
fwd 4096 1280 1280
dgrad 4096 1280 1280
fwd 4096 10240 1280
dgrad 4096 1280 5120
wgrad 1280 1280 4096
wgrad 10240 1280 4096
wgrad 1280 5120 4096
fwd 16384 640 640
fwd 16384 5120 640
dgrad 16384 640 2560
wgrad 640 640 16384
EOF
cat $OUT
