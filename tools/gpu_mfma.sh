# MFMA utilisation of one SDXL train step from PMC counters (one pass: 2 SQ + 1 GRBM counters, kernel
# trace only).  usage: bash tools/gpu_mfma.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-mfma}
shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_${TAG}
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d gpurun_out/pmc_${TAG} -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-vae "$@" \
  > gpurun_out/pmc_${TAG}.log 2>&1 || { echo "mfma pass failed"; tail -20 gpurun_out/pmc_${TAG}.log; exit 1; }
python3 tools/pmc_mfma.py gpurun_out/pmc_${TAG} gpurun_out/pmc_${TAG}.json > /dev/null && rm -rf gpurun_out/pmc_${TAG} && head -c 3000 gpurun_out/pmc_${TAG}.json
