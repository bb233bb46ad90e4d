# One GPU call: train-step parity (incl. graph == eager) -> bench -> LoRA bench.  usage: bash tools/gpu_graph.sh <tag>
set -o pipefail
TAG=${1:-graph}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_train_step_gpu.py tests/test_kernels_gpu.py tests/test_lora_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-vae > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 400 python -u bench.py --model sdxl-lora --steps 14 --warmup 3 > gpurun_out/bench_lora_$TAG.json 2> gpurun_out/bench_lora_$TAG.err || { echo "lora bench failed"; tail -30 gpurun_out/bench_lora_$TAG.err; exit 1; }
cat gpurun_out/bench_lora_$TAG.json
