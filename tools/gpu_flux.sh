set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_flux_gpu.py tests/test_vae_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_flux.log 2>&1 || { echo "pytest failed"; tail -80 gpurun_out/pytest_flux.log; exit 1; }
grep -E "passed|failed|rel err|cosines|losses" gpurun_out/pytest_flux.log | tail -20
