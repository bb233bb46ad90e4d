set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_a6.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_a6.log; exit 1; }
tail -1 gpurun_out/pytest_a6.log
timeout -k 10 200 python -u tools/attn_bench.py | tail -2
