# Attention iteration: parity (test_kernels_gpu -k attention) -> kernel timings, this build vs libotamd_old.so.
# usage: bash tools/gpu_attn.sh <tag>
set -o pipefail
TAG=${1:-attn}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
echo "== new"
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_$TAG.jsonl 2>&1 || { echo "bench failed"; tail -20 gpurun_out/attn_$TAG.jsonl; exit 1; }
cat gpurun_out/attn_$TAG.jsonl
if [ -f onetrainer_amd/_lib/libotamd_old.so ]; then
  echo "== OTAMD_LIB_ALT=old"
  OTAMD_LIB_ALT=old timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_${TAG}_old.jsonl 2>&1 || { echo "bench old failed"; tail -20 gpurun_out/attn_${TAG}_old.jsonl; exit 1; }
  cat gpurun_out/attn_${TAG}_old.jsonl
fi
