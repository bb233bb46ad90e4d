# end of round 4, final tree after the weight-gradient plan changes: the whole -m gpu suite, the smoke, the
# driver-default bench line, a timed-step kernel trace (kstats + stream timeline), SD 1.5 / FLUX lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_fullsize_gpu.py tests/test_flux_gpu.py tests/test_vae_gpu.py tests/test_dp_gpu.py tests/test_bench_gpu.py tests/test_cli_gpu.py > gpurun_out/r4final2_tests_1.log 2>&1; rc1=$?
tail -1 gpurun_out/r4final2_tests_1.log
[ $rc1 -eq 124 ] || [ $rc1 -eq 137 ] || [ $rc1 -eq 134 ] || [ $rc1 -eq 139 ] && { echo "suite 1 died rc=$rc1"; exit 1; }
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ --ignore=tests/test_fullsize_gpu.py --ignore=tests/test_flux_gpu.py --ignore=tests/test_vae_gpu.py --ignore=tests/test_dp_gpu.py --ignore=tests/test_bench_gpu.py --ignore=tests/test_cli_gpu.py > gpurun_out/r4final2_tests_2.log 2>&1; rc2=$?
tail -1 gpurun_out/r4final2_tests_2.log
[ $rc2 -eq 124 ] || [ $rc2 -eq 137 ] || [ $rc2 -eq 134 ] || [ $rc2 -eq 139 ] && { echo "suite 2 died rc=$rc2"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final2_smoke.log 2>&1; rc3=$?
echo "rc suite1=$rc1 suite2=$rc2 smoke=$rc3"
[ $rc1 -eq 0 ] && [ $rc2 -eq 0 ] && [ $rc3 -eq 0 ] || { grep -h -E "FAILED|ERROR" gpurun_out/r4final2_tests_*.log | head; exit 1; }
timeout -k 10 420 python -u bench.py > gpurun_out/r4final2_bench_sdxl_default.json 2> gpurun_out/r4final2_bench_sdxl_default.err || { tail -20 gpurun_out/r4final2_bench_sdxl_default.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4final2_bench_sdxl_default.json')); print('sdxl', d['value'], d['ms_per_step'], d['step_ms_p50'], d['roofline']['frac'], d['roofline']['step_frac'])"
rm -rf gpurun_out/prof_r4f2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4f2 -o run -- python3 -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-vae > gpurun_out/prof_r4f2.log 2>&1 || { tail -30 gpurun_out/prof_r4f2.log; exit 1; }
DB=$(find gpurun_out/prof_r4f2 -name '*.db' | head -1)
python3 tools/prof_summary.py "$DB" gpurun_out/r4final2_kstats_sdxl.csv --steps-kernel adamw_bf16 --top 30 > gpurun_out/r4final2_kstats_sdxl.log 2>&1; head -5 gpurun_out/r4final2_kstats_sdxl.log
python3 tools/timeline.py "$DB" > gpurun_out/r4final2_timeline_sdxl.txt 2>&1; head -8 gpurun_out/r4final2_timeline_sdxl.txt
find gpurun_out/prof_r4f2 -name '*kernel_stats.csv' -exec cp {} gpurun_out/r4final2_rocprof_stats_sdxl.csv \; || true
rm -rf gpurun_out/prof_r4f2
for M in sd15 flux; do
  timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae > gpurun_out/r4final2_bench_$M.json 2> gpurun_out/r4final2_bench_$M.err || { tail -20 gpurun_out/r4final2_bench_$M.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4final2_bench_$M.json')); print('$M', d['value'], d['ms_per_step'], d.get('step_ms_p50'), d['roofline']['frac'])"
done
