# One GPU call: norm parity tests -> LoRA GEMM census -> SDXL bench.  usage: bash tools/gpu_ln.sh <tag>
set -o pipefail
TAG=${1:-ln}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
OTAMD_WGRAD_STREAM=0 timeout -k 10 300 python -u tools/gemm_census.py --steps 2 --lora 32 > gpurun_out/census_lora_$TAG.jsonl 2> gpurun_out/census_lora_$TAG.err || { echo "census failed"; tail -30 gpurun_out/census_lora_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-vae > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
