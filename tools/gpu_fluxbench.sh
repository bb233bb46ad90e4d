set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_flux_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_flux.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_flux.log; exit 1; }
tail -2 gpurun_out/pytest_flux.log
timeout -k 10 500 python -u bench.py --model flux --steps 6 --warmup 2 > gpurun_out/bench_flux.json 2> gpurun_out/bench_flux.err || { echo "bench failed"; tail -30 gpurun_out/bench_flux.err; exit 1; }
cat gpurun_out/bench_flux.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_flux -o run -- python -u bench.py --model flux --steps 3 --warmup 1 > gpurun_out/prof_flux.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_flux.log; exit 1; }
