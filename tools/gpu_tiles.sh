# One GPU call: GEMM parity (all tiles) -> tile/split probe over the SDXL step's GEMMs.  usage: bash tools/gpu_tiles.sh <tag>
set -o pipefail
TAG=${1:-tiles}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 500 python -u tools/gemm_tiles.py --top 18 > gpurun_out/tiles_$TAG.jsonl 2> gpurun_out/tiles_$TAG.err || { echo "probe failed"; tail -30 gpurun_out/tiles_$TAG.err; exit 1; }
cat gpurun_out/tiles_$TAG.jsonl | cut -c1-330
