# One config's bench line + rocprofv3 kernel trace of a short run -> timed-step kernel stats and the
# per-stream timeline (busy time by kernel category, join analysis).
# usage: bash tools/gpu_profile.sh <tag> <model> [extra bench args]
set -o pipefail
TAG=$1; M=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
case $M in sdxl-lora|flux) SK=adamw_f32;; *) SK=adamw_bf16;; esac
timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae "$@" > gpurun_out/bench_${TAG}_$M.json 2> gpurun_out/bench_${TAG}_$M.err || { echo "bench $M failed"; tail -30 gpurun_out/bench_${TAG}_$M.err; exit 1; }
cat gpurun_out/bench_${TAG}_$M.json
rm -rf gpurun_out/prof_${TAG}_$M
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$M -o run -- python -u bench.py --model $M --steps 6 --warmup 2 --no-cpu-baseline --no-vae "$@" > gpurun_out/prof_${TAG}_$M.log 2>&1 || { echo "rocprof $M failed"; tail -30 gpurun_out/prof_${TAG}_$M.log; exit 1; }
DB=$(find gpurun_out/prof_${TAG}_$M -name '*.db' | head -1)
python tools/prof_summary.py "$DB" gpurun_out/kstats_${TAG}_$M.csv --steps-kernel $SK --top 40 > gpurun_out/kstats_${TAG}_$M.log 2>&1 || true
python tools/timeline.py "$DB" --marker $SK --top 25 > gpurun_out/timeline_${TAG}_$M.txt 2>&1 || true
rm -rf gpurun_out/prof_${TAG}_$M
head -20 gpurun_out/timeline_${TAG}_$M.txt
