set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_step_gpu.py tests/test_flux_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_a8.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_a8.log; exit 1; }
tail -1 gpurun_out/pytest_a8.log
bash tools/gpu_ab.sh a8 "OTAMD_LIB_ALT=old" "OTAMD_NOOP=1" 2
