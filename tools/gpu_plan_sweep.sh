# Bench the SDXL step under several OTAMD_GEMM_PLAN overrides (one process each), baseline first and last.
# usage: bash tools/gpu_plan_sweep.sh <tag> "<plan1>" "<plan2>" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
run() {
  OTAMD_GEMM_PLAN="$1" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 12 --warmup 3 > gpurun_out/sweep_${TAG}.json 2> gpurun_out/sweep_${TAG}.err || { echo "bench failed: $1"; tail -5 gpurun_out/sweep_${TAG}.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep_${TAG}.json')); print(round(d['step_ms_p50'],2), round(d['ms_per_step'],2), d['roofline']['achieved'], '|', '$1')"
}
run "" || exit 1
for p in "$@"; do run "$p" || exit 1; done
run "" || exit 1
