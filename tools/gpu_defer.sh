# Deferred split-K reduce milestone: its bitwise tests + the stream-hazard tests, then a same-box A/B of the
# SDXL LoRA bench line (OTAMD_DEFER_REDUCE=0 / 1) and a kernel-stats trace of the deferred run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_defer_reduce_gpu.py tests/test_stream_hazards_gpu.py > gpurun_out/defer_tests.log 2>&1 || { tail -40 gpurun_out/defer_tests.log; exit 1; }
grep -E "deferred reduces|passed|failed" gpurun_out/defer_tests.log
for d in 0 1 0 1; do
  OTAMD_DEFER_REDUCE=$d timeout -k 10 300 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae > gpurun_out/defer_bench_$d.json 2> gpurun_out/defer_bench_$d.err || { tail -20 gpurun_out/defer_bench_$d.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/defer_bench_$d.json')); print('defer=$d', d['value'], d['ms_per_step'], d.get('step_ms_p50'))" | tee -a gpurun_out/defer_ab.txt
done
P=gpurun_out/prof_defer; rm -rf $P
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P -o run -- python3 -u bench.py --model sdxl-lora --steps 6 --warmup 2 --no-cpu-baseline --no-vae > $P.log 2>&1 || { tail -30 $P.log; exit 1; }
DB=$(find $P -name '*.db' | head -1)
python3 tools/prof_summary.py "$DB" gpurun_out/defer_kstats_lora.csv --steps-kernel adamw_bf16 --top 30 > gpurun_out/defer_kstats_lora.log 2>&1; head -12 gpurun_out/defer_kstats_lora.log
python3 tools/timeline.py "$DB" > gpurun_out/defer_timeline_lora.txt 2>&1; head -8 gpurun_out/defer_timeline_lora.txt
rm -rf $P $P.log
