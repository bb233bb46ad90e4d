# A/B on one box: GEMM planner with / without the 128x128 tile, alternating runs.  usage: bash tools/gpu_ab_t4.sh <tag>
set -o pipefail
TAG=${1:-t4}
export TMPDIR=/tmp
mkdir -p gpurun_out
for R in 1 2; do for V in 0 1; do
  OTAMD_GEMM_NO_T4=$V timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 20 --warmup 4 > gpurun_out/ab_${TAG}_${R}_${V}.json 2> gpurun_out/ab_${TAG}_${R}_${V}.err || { echo "bench failed"; tail -20 gpurun_out/ab_${TAG}_${R}_${V}.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_${R}_${V}.json')); print('run $R no_t4 $V', d['value'], d['step_ms_p50'], d['roofline']['achieved'])"
done; done
