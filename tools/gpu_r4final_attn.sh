set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/kp_r4h2
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kp_r4h2 -o run -- python3 -u tools/attn_bench.py --reps 10 > gpurun_out/kp_r4h2.log 2>&1 || { tail -20 gpurun_out/kp_r4h2.log; exit 1; }
python3 tools/ktrace_by_grid.py gpurun_out/kp_r4h2 --match attn --top 40 | tee gpurun_out/r4final_attn_by_grid.txt
rm -rf gpurun_out/kp_r4h2
