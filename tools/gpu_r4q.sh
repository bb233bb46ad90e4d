# mid-round 4 SDXL state: bench line, timed-step kernel stats + stream timeline (kernel trace only), GEMM census
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --no-cpu-baseline --no-vae > gpurun_out/r4q_bench.json 2> gpurun_out/r4q_bench.err || { tail -30 gpurun_out/r4q_bench.err; exit 1; }
cat gpurun_out/r4q_bench.json
rm -rf gpurun_out/prof_r4q
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4q -o run -- python3 -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-vae > gpurun_out/prof_r4q.log 2>&1 || { tail -30 gpurun_out/prof_r4q.log; exit 1; }
DB=$(find gpurun_out/prof_r4q -name '*.db' | head -1)
python3 tools/prof_summary.py "$DB" gpurun_out/r4q_kstats.csv --steps-kernel adamw_bf16 --top 30 > gpurun_out/r4q_kstats.log 2>&1; head -30 gpurun_out/r4q_kstats.log
python3 tools/timeline.py "$DB" > gpurun_out/r4q_timeline.txt 2>&1; head -14 gpurun_out/r4q_timeline.txt
find gpurun_out/prof_r4q -name '*kernel_stats.csv' -exec cp {} gpurun_out/r4q_rocprof_stats.csv \; || true
rm -rf gpurun_out/prof_r4q
timeout -k 10 300 python3 -u tools/gemm_census.py --steps 2 > gpurun_out/r4q_census.jsonl 2> gpurun_out/r4q_census.err || { tail -20 gpurun_out/r4q_census.err; exit 1; }
echo census done
