# end of round 4, part B: the driver-default bench line, a timed-step kernel trace (kstats + stream timeline), the
# GEMM-family PMC traffic of the bench config (what bench.py's roofline.traffic reads), the other configs' lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u bench.py > gpurun_out/r4end_bench_sdxl_default.json 2> gpurun_out/r4end_bench_sdxl_default.err || { tail -20 gpurun_out/r4end_bench_sdxl_default.err; exit 1; }
cat gpurun_out/r4end_bench_sdxl_default.json
rm -rf gpurun_out/prof_r4end
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4end -o run -- python3 -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-vae > gpurun_out/prof_r4end.log 2>&1 || { tail -30 gpurun_out/prof_r4end.log; exit 1; }
DB=$(find gpurun_out/prof_r4end -name '*.db' | head -1)
python3 tools/prof_summary.py "$DB" gpurun_out/r4end_kstats_sdxl.csv --steps-kernel adamw_bf16 --top 30 > gpurun_out/r4end_kstats_sdxl.log 2>&1; head -12 gpurun_out/r4end_kstats_sdxl.log
python3 tools/timeline.py "$DB" > gpurun_out/r4end_timeline_sdxl.txt 2>&1; head -8 gpurun_out/r4end_timeline_sdxl.txt
find gpurun_out/prof_r4end -name '*kernel_stats.csv' -exec cp {} gpurun_out/r4end_rocprof_stats_sdxl.csv \; || true
rm -rf gpurun_out/prof_r4end
bash tools/gpu_pmc.sh traffic_sdxl > gpurun_out/r4end_pmc.log 2>&1 || { tail -20 gpurun_out/r4end_pmc.log; exit 1; }
tail -5 gpurun_out/r4end_pmc.log
for M in sd15 sdxl-lora flux; do
  timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae > gpurun_out/r4end_bench_$M.json 2> gpurun_out/r4end_bench_$M.err || { tail -20 gpurun_out/r4end_bench_$M.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4end_bench_$M.json')); print('$M', d['value'], d['ms_per_step'], d.get('step_ms_p50'), d['roofline']['frac'])"
done
