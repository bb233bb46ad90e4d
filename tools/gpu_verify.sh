# One GPU call: full GPU parity suite -> census -> bench (FT) -> bench (LoRA C4).  usage: bash tools/gpu_verify.sh <tag>
set -o pipefail
TAG=${1:-verify}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
OTAMD_WGRAD_STREAM=0 timeout -k 10 300 python -u tools/gemm_census.py --steps 2 > gpurun_out/census_$TAG.jsonl 2> gpurun_out/census_$TAG.err || { echo "census failed"; tail -30 gpurun_out/census_$TAG.err; exit 1; }
tail -1 gpurun_out/census_$TAG.jsonl
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-vae > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 400 python -u bench.py --model sdxl-lora --steps 14 --warmup 3 > gpurun_out/bench_lora_$TAG.json 2> gpurun_out/bench_lora_$TAG.err || { echo "lora bench failed"; tail -30 gpurun_out/bench_lora_$TAG.err; exit 1; }
cat gpurun_out/bench_lora_$TAG.json
