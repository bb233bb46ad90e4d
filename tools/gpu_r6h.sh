# Round 6: C4 A/B of the fused LoRA down-projection's size limit (OTAMD_LORA_FUSE_MNK), interleaved x2.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae --steps 15 > gpurun_out/r6h_$name.json 2> gpurun_out/r6h_$name.err || { echo "$name failed"; tail -5 gpurun_out/r6h_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6h_$name.json')); print('$name', d['value'], d['ms_per_step'], d['step_ms_p50'], d['loss'], d['lora_forwards_fused_vs_two_launch'])"
}
for rep in 1 2; do
  run fuse0 OTAMD_LORA_FUSE=0
  run mnk25 OTAMD_LORA_FUSE_MNK=2.5e10
  run mnk8 OTAMD_LORA_FUSE_MNK=8e9
  run mnk60 OTAMD_LORA_FUSE_MNK=6e10
done
