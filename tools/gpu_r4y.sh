# Deterministic grad-norm (per-chunk slots, per-tensor sums in chunk order): optimizer / step / host-layer GPU tests,
# then three identical SDXL bench runs whose losses must agree to the last printed digit
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_optimizer_gpu.py tests/test_train_step_gpu.py tests/test_host_layer_gpu.py > gpurun_out/r4y_tests.log 2>&1 || { tail -40 gpurun_out/r4y_tests.log; exit 1; }
tail -1 gpurun_out/r4y_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-vae > gpurun_out/r4y_bench_$i.json 2> gpurun_out/r4y_bench_$i.err || { tail -20 gpurun_out/r4y_bench_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4y_bench_$i.json')); print('run $i', d['ms_per_step'], d['step_ms_p50'], repr(d['loss']))"
done
