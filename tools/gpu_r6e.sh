# Round 6: upper bound of fusing the LoRA down-projections (t = x A^T, u = dy sB) into the base GEMMs: C4 with the
# t / u GEMMs and their split-K reduces skipped (OTAMD_LORA_FREE_T=1, results garbage) against the real step.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae --steps 15 > gpurun_out/r6e_$name.json 2> gpurun_out/r6e_$name.err || { echo "$name failed"; tail -5 gpurun_out/r6e_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6e_$name.json')); print('$name', d['value'], d['ms_per_step'], d['step_ms_p50'], d['loss'])"
}
for rep in 1 2; do
  run base OTAMD_LORA_FREE_T=0
  run free OTAMD_LORA_FREE_T=1
done
