# end of round 4, part A: the whole -m gpu suite (two pytest processes, each test with its own timeout) and the smoke
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_fullsize_gpu.py tests/test_flux_gpu.py tests/test_vae_gpu.py tests/test_dp_gpu.py tests/test_bench_gpu.py tests/test_cli_gpu.py > gpurun_out/r4end_tests_1.log 2>&1; rc1=$?
tail -3 gpurun_out/r4end_tests_1.log
[ $rc1 -eq 124 ] || [ $rc1 -eq 137 ] || [ $rc1 -eq 134 ] || [ $rc1 -eq 139 ] && { echo "suite 1 died rc=$rc1"; exit 1; }
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ --ignore=tests/test_fullsize_gpu.py --ignore=tests/test_flux_gpu.py --ignore=tests/test_vae_gpu.py --ignore=tests/test_dp_gpu.py --ignore=tests/test_bench_gpu.py --ignore=tests/test_cli_gpu.py > gpurun_out/r4end_tests_2.log 2>&1; rc2=$?
tail -3 gpurun_out/r4end_tests_2.log
[ $rc2 -eq 124 ] || [ $rc2 -eq 137 ] || [ $rc2 -eq 134 ] || [ $rc2 -eq 139 ] && { echo "suite 2 died rc=$rc2"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4end_smoke.log 2>&1; rc3=$?
tail -3 gpurun_out/r4end_smoke.log
echo "rc suite1=$rc1 suite2=$rc2 smoke=$rc3"
grep -h -E "PASSED|FAILED|ERROR" gpurun_out/r4end_tests_1.log gpurun_out/r4end_tests_2.log | grep -c PASSED
grep -h -E "FAILED|ERROR" gpurun_out/r4end_tests_1.log gpurun_out/r4end_tests_2.log | head -20 || true
