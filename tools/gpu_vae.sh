set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vae_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_vae.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_vae.log; exit 1; }
tail -3 gpurun_out/pytest_vae.log
timeout -k 10 200 python -u tools/bench_vae.py > gpurun_out/bench_vae.json 2>&1 || { echo "vae bench failed"; tail -30 gpurun_out/bench_vae.json; exit 1; }
cat gpurun_out/bench_vae.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vae -o run -- python -u tools/bench_vae.py --iters 3 > gpurun_out/prof_vae.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_vae.log; exit 1; }
