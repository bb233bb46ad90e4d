set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_train_step_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_nofix.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_nofix.log; exit 1; }
tail -2 gpurun_out/pytest_nofix.log
bash tools/gpu_ab.sh nofix "OTAMD_LIB_ALT=old" "OTAMD_NOOP=1" 3
