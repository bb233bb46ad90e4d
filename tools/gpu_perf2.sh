# Perf iteration: parity subset -> bench -> rocprof kernel trace of a short bench -> timed-step kernel stats
# + per-stream timeline.  usage: bash tools/gpu_perf2.sh <tag> [pytest selection...]
set -o pipefail
TAG=${1:-perf}
shift || true
SEL=${@:-tests/test_kernels_gpu.py tests/test_train_step_gpu.py tests/test_gemm_gpu.py}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest $SEL -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-vae > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-vae > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
DB=$(find gpurun_out/prof_$TAG -name '*.db' | head -1)
python tools/prof_summary.py "$DB" gpurun_out/kstats_$TAG.csv --top 45 > gpurun_out/kstats_$TAG.log 2>&1 || true
python tools/timeline.py "$DB" > gpurun_out/timeline_$TAG.log 2>&1 || true
rm -rf gpurun_out/prof_$TAG
cat gpurun_out/kstats_$TAG.log | head -50
cat gpurun_out/timeline_$TAG.log
