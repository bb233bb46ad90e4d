# end of round 4 (final tree), part A: the whole -m gpu suite (two pytest processes, each test with its own timeout) and the smoke
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_fullsize_gpu.py tests/test_flux_gpu.py tests/test_vae_gpu.py tests/test_dp_gpu.py tests/test_bench_gpu.py tests/test_cli_gpu.py > gpurun_out/r4final_tests_1.log 2>&1; rc1=$?
tail -3 gpurun_out/r4final_tests_1.log
[ $rc1 -eq 124 ] || [ $rc1 -eq 137 ] || [ $rc1 -eq 134 ] || [ $rc1 -eq 139 ] && { echo "suite 1 died rc=$rc1"; exit 1; }
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ --ignore=tests/test_fullsize_gpu.py --ignore=tests/test_flux_gpu.py --ignore=tests/test_vae_gpu.py --ignore=tests/test_dp_gpu.py --ignore=tests/test_bench_gpu.py --ignore=tests/test_cli_gpu.py > gpurun_out/r4final_tests_2.log 2>&1; rc2=$?
tail -3 gpurun_out/r4final_tests_2.log
[ $rc2 -eq 124 ] || [ $rc2 -eq 137 ] || [ $rc2 -eq 134 ] || [ $rc2 -eq 139 ] && { echo "suite 2 died rc=$rc2"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final_smoke.log 2>&1; rc3=$?
tail -3 gpurun_out/r4final_smoke.log
echo "rc suite1=$rc1 suite2=$rc2 smoke=$rc3"
grep -h -E "PASSED|FAILED|ERROR" gpurun_out/r4final_tests_1.log gpurun_out/r4final_tests_2.log | grep -c PASSED
grep -h -E "FAILED|ERROR" gpurun_out/r4final_tests_1.log gpurun_out/r4final_tests_2.log | head -20 || true
timeout -k 10 420 python -u bench.py > gpurun_out/r4final_bench_sdxl_default.json 2> gpurun_out/r4final_bench_sdxl_default.err || { tail -20 gpurun_out/r4final_bench_sdxl_default.err; exit 1; }
cat gpurun_out/r4final_bench_sdxl_default.json
timeout -k 10 400 python -u bench.py --model flux --no-cpu-baseline --no-vae > gpurun_out/r4final_bench_flux.json 2> gpurun_out/r4final_bench_flux.err || { tail -20 gpurun_out/r4final_bench_flux.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4final_bench_flux.json')); print('flux', d['value'], d['ms_per_step'], d.get('step_ms_p50'), d['roofline']['frac'])"
