# Round 6: C4 with the fused LoRA input gradient (single-module + q|k|v sites) on vs off, 3 interleaved rounds
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2 3; do
  for v in 1 0; do
    OTAMD_LORA_FUSE_DGRAD=$v timeout -k 10 400 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae > gpurun_out/r6ag_${v}_$r.json 2> gpurun_out/r6ag.err || { tail -20 gpurun_out/r6ag.err; exit 1; }
  done
  python3 -c "
import json
a=json.load(open('gpurun_out/r6ag_1_$r.json')); b=json.load(open('gpurun_out/r6ag_0_$r.json'))
print('fused', a['ms_per_step'], a['step_ms_p50'], 'two-launch', b['ms_per_step'], b['step_ms_p50'])"
done
