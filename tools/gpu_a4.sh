set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_attn.sh a4 || exit 1
timeout -k 10 400 python -u tools/gemm_census.py --flux --steps 1 > gpurun_out/census_flux.jsonl 2> gpurun_out/census_flux.err || { echo "census failed"; tail -20 gpurun_out/census_flux.err; exit 1; }
head -25 gpurun_out/census_flux.jsonl; tail -1 gpurun_out/census_flux.jsonl
