# One GPU call: GEMM + kernel + step parity -> tile probe -> census -> bench.  usage: bash tools/gpu_tiles2.sh <tag>
set -o pipefail
TAG=${1:-tiles2}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_train_step_gpu.py tests/test_unet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 500 python -u tools/gemm_tiles.py --top 24 > gpurun_out/tiles_$TAG.jsonl 2> gpurun_out/tiles_$TAG.err || { echo "probe failed"; tail -30 gpurun_out/tiles_$TAG.err; exit 1; }
grep mismatch gpurun_out/tiles_$TAG.err | head -20
OTAMD_WGRAD_STREAM=0 timeout -k 10 300 python -u tools/gemm_census.py --steps 2 > gpurun_out/census_$TAG.jsonl 2> gpurun_out/census_$TAG.err || { echo "census failed"; tail -30 gpurun_out/census_$TAG.err; exit 1; }
tail -1 gpurun_out/census_$TAG.jsonl
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-vae > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
