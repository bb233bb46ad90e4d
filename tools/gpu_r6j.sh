# Round 6: FLUX adapter weight-gradient shapes (MN x MN, M or N = rank 16, K = tokens) alone, table plan vs others.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for sp in "wgrad:16:3072:9216 6:16,6:8,6:32,5:16,4:16" "wgrad:16:12288:9216 6:5,6:10,6:2,5:5,4:5" \
          "wgrad:16:15360:9524 6:4,6:8,6:2,5:4,4:4" "wgrad:3072:16:9216 6:10,5:10,5:20,6:20,4:10" \
          "wgrad:3072:16:9524 5:15,5:8,5:30,6:15" "wgrad:12288:16:9524 4:5,5:5,5:2,5:10,6:5" "wgrad:64:3072:9524 6:10,6:5,6:20,5:10"; do
  set -- $sp
  timeout -k 10 120 python -u tools/gemm_tile_sweep.py --shapes $1 --plans $2 --reps 20 >> gpurun_out/r6_flux_wgrad_sweep.jsonl 2>> gpurun_out/r6_flux_wgrad_sweep.err || { tail -5 gpurun_out/r6_flux_wgrad_sweep.err; exit 1; }
done
cat gpurun_out/r6_flux_wgrad_sweep.jsonl
