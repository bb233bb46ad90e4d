# same-box A/B of the GEMM K-loop schedule on the SDXL step: OTAMD_GEMM_HK=0 (whole K-tile DMA) vs 2 (half-K units for
# the weight gradients) vs 1 (half-K units everywhere), interleaved
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2; do for v in 0 2 1; do
  OTAMD_GEMM_HK=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 15 --warmup 4 $BENCH_ARGS > gpurun_out/abhk_${v}_$rep.json 2> gpurun_out/abhk_${v}_$rep.err || { tail -5 gpurun_out/abhk_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/abhk_${v}_$rep.json')); print('HK=$v', d['ms_per_step'], d['step_ms_p50'], d['loss'], d['roofline']['frac'])"
done; done
