# Round 6: C4 run-to-run loss check -- native host layer, ctypes host path (OTAMD_HOST=0), and the ctypes path with
# the fused LoRA down-projection off.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae --steps 8 --warmup 3 > gpurun_out/r6m_$name.json 2> gpurun_out/r6m_$name.err || { echo "$name failed"; tail -5 gpurun_out/r6m_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6m_$name.json')); print('$name', d['ms_per_step'], repr(d['loss']), d['lora_forwards_fused_vs_two_launch'])"
}
for rep in 1 2 3; do
  run native OTAMD_HOST=1
  run ctypes OTAMD_HOST=0
  run ctypes_nofuse OTAMD_HOST=0 OTAMD_LORA_FUSE=0
  run native_nofuse OTAMD_HOST=1 OTAMD_LORA_FUSE=0
done
