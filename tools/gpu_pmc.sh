# HBM traffic of one SDXL train step from PMC counters: two separate rocprofv3 passes (FETCH_SIZE, then
# WRITE_SIZE: they do not fit one TCC pass), counters only with the kernel trace.
# usage: bash tools/gpu_pmc.sh <tag> [bench args, e.g. --model sd15]
set -o pipefail
TAG=${1:-pmc}
shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_${TAG}_$C
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_$C -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-vae "$@" > gpurun_out/pmc_${TAG}_$C.log 2>&1 || { echo "pmc pass $C failed"; tail -20 gpurun_out/pmc_${TAG}_$C.log; exit 1; }
  find gpurun_out/pmc_${TAG}_$C -name '*.csv' | head
done
python3 tools/pmc_traffic.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE > gpurun_out/pmc_${TAG}.json && rm -rf gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE && cat gpurun_out/pmc_${TAG}.json
