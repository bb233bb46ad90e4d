# Bench line + timed-step rocprof kernel stats for BASELINE configs.  usage: bash tools/gpu_configs.sh <tag> <model>...
# (model: sdxl | sd15 | sdxl-lora | flux; the optimizer kernel that marks step boundaries is picked per model)
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for M in "$@"; do
  case $M in sdxl-lora|flux) SK=adamw_f32;; *) SK=adamw_bf16;; esac
  timeout -k 10 500 python -u bench.py --model $M --no-cpu-baseline --no-vae > gpurun_out/bench_${TAG}_$M.json 2> gpurun_out/bench_${TAG}_$M.err || { echo "bench $M failed"; tail -30 gpurun_out/bench_${TAG}_$M.err; exit 1; }
  cat gpurun_out/bench_${TAG}_$M.json
  rm -rf gpurun_out/prof_${TAG}_$M
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$M -o run -- python -u bench.py --model $M --steps 6 --warmup 2 --no-cpu-baseline --no-vae > gpurun_out/prof_${TAG}_$M.log 2>&1 || { echo "rocprof $M failed"; tail -30 gpurun_out/prof_${TAG}_$M.log; exit 1; }
  DB=$(find gpurun_out/prof_${TAG}_$M -name '*.db' | head -1)
  python tools/prof_summary.py "$DB" gpurun_out/kstats_${TAG}_$M.csv --steps-kernel $SK --top 30 > gpurun_out/kstats_${TAG}_$M.log 2>&1 || true
  find gpurun_out/prof_${TAG}_$M -name '*kernel_stats.csv' -exec cp {} gpurun_out/rocprof_stats_${TAG}_$M.csv \; || true
  rm -rf gpurun_out/prof_${TAG}_$M
  head -12 gpurun_out/kstats_${TAG}_$M.log
done
