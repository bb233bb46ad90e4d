# Round 6: fused conv LoRA forward (OTAMD_LORA_FUSE_CONV=1) vs two launches on the final tree, C4, 2 pairs
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  for v in 1 0; do
    OTAMD_LORA_FUSE_CONV=$v timeout -k 10 400 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae > gpurun_out/r6aq_${v}_$r.json 2> gpurun_out/r6aq.err || { tail -20 gpurun_out/r6aq.err; exit 1; }
  done
  python3 -c "
import json
a=json.load(open('gpurun_out/r6aq_1_$r.json')); b=json.load(open('gpurun_out/r6aq_0_$r.json'))
print('conv fused', a['ms_per_step'], a['step_ms_p50'], 'two-launch', b['ms_per_step'], b['step_ms_p50'])"
done
