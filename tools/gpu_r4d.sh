# round 4: where the SDXL step's time goes -- kernel trace + HIP runtime trace of timed steps (gap causes, stream
# timeline, per-kernel stats) and the in-step GEMM census by stream
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_r4d
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/prof_r4d -o run -- python3 -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-vae > gpurun_out/prof_r4d.log 2>&1 || { tail -30 gpurun_out/prof_r4d.log; exit 1; }
DB=$(find gpurun_out/prof_r4d -name '*.db' | head -1)
python3 tools/gap_causes.py "$DB" --top 30 > gpurun_out/r4d_gaps.txt 2>&1; cat gpurun_out/r4d_gaps.txt
python3 tools/timeline.py "$DB" > gpurun_out/r4d_timeline.txt 2>&1; head -12 gpurun_out/r4d_timeline.txt
python3 tools/prof_summary.py "$DB" gpurun_out/r4d_kstats.csv --steps-kernel adamw_bf16 --top 30 > gpurun_out/r4d_kstats.log 2>&1; head -30 gpurun_out/r4d_kstats.log
rm -rf gpurun_out/prof_r4d
timeout -k 10 300 python3 -u tools/gemm_census.py --steps 2 > gpurun_out/r4d_census.jsonl 2> gpurun_out/r4d_census.err || { tail -20 gpurun_out/r4d_census.err; exit 1; }
head -40 gpurun_out/r4d_census.jsonl
