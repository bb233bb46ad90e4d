set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_gpu.py tests/test_train_step_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sd15.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_sd15.log; exit 1; }
tail -3 gpurun_out/pytest_sd15.log
timeout -k 10 300 python -u bench.py --model sd15 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_sd15.json 2> gpurun_out/bench_sd15.err || { echo "bench failed"; tail -30 gpurun_out/bench_sd15.err; exit 1; }
cat gpurun_out/bench_sd15.json
