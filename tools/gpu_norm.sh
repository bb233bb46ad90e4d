set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_gpu.py tests/test_train_step_gpu.py tests/test_vae_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_norm.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_norm.log; exit 1; }
tail -2 gpurun_out/pytest_norm.log
timeout -k 10 300 python -u tools/hbm_bench.py --only gn,ln > gpurun_out/hbm_norm.log 2>&1 || { echo "hbm failed"; tail -20 gpurun_out/hbm_norm.log; exit 1; }
grep -v amdgpu gpurun_out/hbm_norm.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-vae > gpurun_out/bench_norm.json 2> gpurun_out/bench_norm.err || { echo "bench failed"; tail -30 gpurun_out/bench_norm.err; exit 1; }
cat gpurun_out/bench_norm.json
