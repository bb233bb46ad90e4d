# One GPU call: parity suite -> bench -> rocprof kernel-trace of a short bench.  Stops at the first failure.
# usage: bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-run}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-vae > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG -name '*.csv' -o -name '*.db' | head
