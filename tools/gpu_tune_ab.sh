# One GPU call: SDXL bench with the analytic GEMM plans vs plans autotuned in the warm-up (with and
# without the 160-wide tiles).  usage: bash tools/gpu_tune_ab.sh <tag>
set -o pipefail
TAG=${1:-tune}
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-vae --steps 15 "$@" > gpurun_out/ab_${TAG}_$n.json 2> gpurun_out/ab_${TAG}_$n.err || { echo "$n failed"; tail -20 gpurun_out/ab_${TAG}_$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_$n.json')); print('$n', d['value'], d['ms_per_step'], d['step_ms_p50'], d['roofline']['achieved'])"
}
run analytic
OTAMD_TUNE_TILES=0,1,2,3,4,5,6,-1 run tuned_old --autotune
run tuned_all --autotune
run analytic2
