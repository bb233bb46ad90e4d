set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_optimizer_gpu.py tests/test_train_step_gpu.py tests/test_cli_gpu.py tests/test_dp_gpu.py tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_defer_reduce_gpu.py > gpurun_out/r6a_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6a_tests.log; grep -E "FAILED|ERROR" gpurun_out/r6a_tests.log | head -20
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err || { tail -20 gpurun_out/r6a_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6a_bench.json')); print('sdxl', d['value'], d['ms_per_step'], d['step_ms_p50'], d['roofline']['frac'], d['roofline']['step_frac'])"
