# End-of-round / milestone GPU run, one box: the whole -m gpu suite (two halves, each under its own limit), the
# smoke, the driver-default bench line (CPU baseline + VAE), a rocprofv3 kernel trace of timed steps (kernel stats
# + stream timeline) and the SD 1.5 / FLUX lines.   usage: bash tools/gpu_suite.sh <tag> [--no-tests] [--no-extra]
set -o pipefail
TAG=${1:?tag}; shift
TESTS=1; EXTRA=1
for a in "$@"; do case $a in --no-tests) TESTS=0;; --no-extra) EXTRA=0;; esac; done
mkdir -p gpurun_out
export TMPDIR=/tmp
dead() { [ $1 -eq 124 ] || [ $1 -eq 137 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
if [ $TESTS = 1 ]; then
  HEAVY="tests/test_fullsize_gpu.py tests/test_flux_gpu.py tests/test_vae_gpu.py tests/test_dp_gpu.py tests/test_bench_gpu.py tests/test_cli_gpu.py"
  timeout -k 10 560 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu $HEAVY > gpurun_out/${TAG}_tests_1.log 2>&1; rc1=$?
  tail -1 gpurun_out/${TAG}_tests_1.log; dead $rc1 && { echo "suite 1 died rc=$rc1"; exit 1; }
  IGN=$(for f in $HEAVY; do printf -- "--ignore=%s " $f; done)
  timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ $IGN > gpurun_out/${TAG}_tests_2.log 2>&1; rc2=$?
  tail -1 gpurun_out/${TAG}_tests_2.log; dead $rc2 && { echo "suite 2 died rc=$rc2"; exit 1; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc3=$?
  echo "rc suite1=$rc1 suite2=$rc2 smoke=$rc3"
  [ $rc1 -eq 0 ] && [ $rc2 -eq 0 ] && [ $rc3 -eq 0 ] || { grep -h -E "FAILED|ERROR" gpurun_out/${TAG}_tests_*.log | head; exit 1; }
fi
timeout -k 10 420 python -u bench.py > gpurun_out/${TAG}_bench_sdxl_default.json 2> gpurun_out/${TAG}_bench_sdxl_default.err || { tail -20 gpurun_out/${TAG}_bench_sdxl_default.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_sdxl_default.json')); print('sdxl', d['value'], d['ms_per_step'], d['step_ms_p50'], d['roofline']['frac'], d['roofline']['step_frac'])"
P=gpurun_out/prof_$TAG; rm -rf $P
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P -o run -- python3 -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-vae > $P.log 2>&1 || { tail -30 $P.log; exit 1; }
DB=$(find $P -name '*.db' | head -1)
python3 tools/prof_summary.py "$DB" gpurun_out/${TAG}_kstats_sdxl.csv --steps-kernel adamw_bf16 --top 30 > gpurun_out/${TAG}_kstats_sdxl.log 2>&1; head -5 gpurun_out/${TAG}_kstats_sdxl.log
python3 tools/timeline.py "$DB" > gpurun_out/${TAG}_timeline_sdxl.txt 2>&1; head -8 gpurun_out/${TAG}_timeline_sdxl.txt
find $P -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_rocprof_stats_sdxl.csv \; || true
rm -rf $P $P.log
if [ $EXTRA = 1 ]; then
  for M in sd15 flux sdxl-lora; do
    timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae > gpurun_out/${TAG}_bench_$M.json 2> gpurun_out/${TAG}_bench_$M.err || { tail -20 gpurun_out/${TAG}_bench_$M.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_$M.json')); print('$M', d['value'], d['ms_per_step'], d.get('step_ms_p50'), d['roofline']['frac'])"
  done
fi
