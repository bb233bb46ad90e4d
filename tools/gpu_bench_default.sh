# The driver's default bench line (N=1, incl. the CPU baseline), then the Flux LoRA line.  usage: bash tools/gpu_bench_default.sh <tag>
set -o pipefail
TAG=${1:-def}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_${TAG}_default.json 2> gpurun_out/bench_${TAG}_default.err || { echo "bench failed"; tail -30 gpurun_out/bench_${TAG}_default.err; exit 1; }
cat gpurun_out/bench_${TAG}_default.json
