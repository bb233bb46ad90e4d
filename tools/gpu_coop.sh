# One GPU call: coop split-K parity -> GEMM parity -> tile probe (with coop candidate) -> bench A/B (OTAMD_GEMM_SK=0 vs 1)
# usage: bash tools/gpu_coop.sh <tag>
set -o pipefail
TAG=${1:-coop}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_coop_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_coop_$TAG.log 2>&1 || { echo "coop pytest failed"; tail -60 gpurun_out/pytest_coop_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_coop_$TAG.log
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_train_step_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 500 python -u tools/gemm_tiles.py --top 24 > gpurun_out/tiles_$TAG.jsonl 2> gpurun_out/tiles_$TAG.err || { echo "probe failed"; tail -30 gpurun_out/tiles_$TAG.err; exit 1; }
grep mismatch gpurun_out/tiles_$TAG.err | head -20
bash tools/gpu_ab.sh $TAG "OTAMD_GEMM_SK=0" "OTAMD_GEMM_SK=1" 2
