# Round 6: GEMM census of the SDXL step at HEAD, then the overlapped-AdamW A/B (grid caps).
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_census.py --steps 2 > gpurun_out/r6_gemm_census_sdxl.jsonl 2> gpurun_out/r6_gemm_census_sdxl.err || { tail -20 gpurun_out/r6_gemm_census_sdxl.err; exit 1; }
tail -1 gpurun_out/r6_gemm_census_sdxl.jsonl
bash tools/gpu_ab_optoverlap.sh r6opt 128 256 512
