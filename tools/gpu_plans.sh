# One GPU call: build the measured GEMM plan table (onetrainer_amd/gemm_plans_mi355x.json) by autotuning
# every GEMM signature inside the real train steps of the benchmarked configurations, then bench SDXL
# with the table (the default) against the analytic planner.  usage: bash tools/gpu_plans.sh <tag> [models...]
set -o pipefail
TAG=${1:-plans}; shift
MODELS=${@:-sdxl sd15 sdxl-lora flux}
export TMPDIR=/tmp OTAMD_TUNE_REPS=5
mkdir -p gpurun_out
OUT=gpurun_out/gemm_plans_mi355x.json
rm -f $OUT
for m in $MODELS; do
  timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline --no-vae --steps 6 --warmup 4 --autotune --dump-plans $OUT > gpurun_out/plans_${TAG}_$m.json 2> gpurun_out/plans_${TAG}_$m.err || { echo "$m failed"; tail -20 gpurun_out/plans_${TAG}_$m.err; exit 1; }
  tail -1 gpurun_out/plans_${TAG}_$m.err
done
cp $OUT onetrainer_amd/gemm_plans_mi355x.json
for m in $MODELS; do
  for v in table analytic; do
    E=1; [ $v = analytic ] && E=0
    OTAMD_GEMM_TABLE=$E timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline --no-vae --steps 15 > gpurun_out/plans_${TAG}_${m}_$v.json 2> gpurun_out/plans_${TAG}_${m}_$v.err || { echo "$m $v failed"; tail -20 gpurun_out/plans_${TAG}_${m}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/plans_${TAG}_${m}_$v.json')); print('$m $v', d['value'], d['ms_per_step'], d['step_ms_p50'], d['gemm_plans'])"
  done
done
