set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_a7.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_a7.log; exit 1; }
OTAMD_ATTN_FWD64_W4=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_a7b.log 2>&1 || { echo "pytest W4 failed"; tail -40 gpurun_out/pytest_a7b.log; exit 1; }
tail -1 gpurun_out/pytest_a7.log
timeout -k 10 200 python -u tools/attn_bench.py
OTAMD_ATTN_FWD64_W4=1 timeout -k 10 200 python -u tools/attn_bench.py
