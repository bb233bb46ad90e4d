# Round 6: C4 timed-step kernel trace at HEAD (kernel stats + stream timeline)
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
P=gpurun_out/prof_r6k; rm -rf $P
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P -o run -- python3 -u bench.py --model sdxl-lora --steps 8 --warmup 2 --no-cpu-baseline --no-vae > $P.log 2>&1 || { tail -30 $P.log; exit 1; }
DB=$(find $P -name '*.db' | head -1)
python3 tools/prof_summary.py "$DB" gpurun_out/r6k_kstats_sdxl-lora.csv --steps-kernel adamw_f32 --top 40 > gpurun_out/r6k_kstats_sdxl-lora.log 2>&1; head -5 gpurun_out/r6k_kstats_sdxl-lora.log
python3 tools/timeline.py "$DB" --marker adamw_f32 > gpurun_out/r6k_timeline_sdxl-lora.txt 2>&1; head -48 gpurun_out/r6k_timeline_sdxl-lora.txt
rm -rf $P $P.log
