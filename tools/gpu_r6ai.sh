# Round 6: fused-LoRA tile table variants on C4: all entries (1), fused-tile entries only (2), none (0); 2 rounds
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  for v in 1 2 0; do
    OTAMD_LORA_PLANS=$v timeout -k 10 400 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae > gpurun_out/r6ai_${v}_$r.json 2> gpurun_out/r6ai.err || { tail -20 gpurun_out/r6ai.err; exit 1; }
    python3 -c "
import json
a=json.load(open('gpurun_out/r6ai_${v}_$r.json'))
print('plans=$v', a['ms_per_step'], a['step_ms_p50'], a['step_ms_p90'], a['step_ms_max'], a['lora_forwards_fused_vs_two_launch'])"
  done
done
