# Round 6: LoRA configs (C5 FLUX, C4 SDXL) with the weight-gradient side stream on (default) and off
# (OTAMD_WGRAD_STREAM=0: the adapter weight gradients in line on the main stream), interleaved x2.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
run() {  # model, name, env...
  local m=$1 name=$2; shift 2
  env "$@" timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline --no-vae --steps 12 > gpurun_out/r6k_${m}_$name.json 2> gpurun_out/r6k_${m}_$name.err || { echo "$m $name failed"; tail -5 gpurun_out/r6k_${m}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6k_${m}_$name.json')); print('$m $name', d['value'], d['ms_per_step'], d['step_ms_p50'], d['loss'])"
}
for rep in 1 2; do
  for m in flux sdxl-lora; do
    run $m side OTAMD_WGRAD_STREAM=1
    run $m inline OTAMD_WGRAD_STREAM=0
  done
done
