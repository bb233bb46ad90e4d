# SDXL LoRA (C4): the rank-32 adapter weight gradients (side stream) with split-K capped at 4 / 2 against the table
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp OTAMD_HOST=0
for rep in 1 2; do
  for arm in none x2; do
    case $arm in none) P="";; x2) P=$(cat ab_tables/lora_x2.txt);; esac
    OTAMD_GEMM_PLAN="$P" timeout -k 10 300 python -u bench.py --model sdxl-lora --steps 15 --no-cpu-baseline --no-vae > gpurun_out/r4lora_$arm.json 2> gpurun_out/r4lora_$arm.err || { tail -5 gpurun_out/r4lora_$arm.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4lora_$arm.json')); print('$arm', d['value'], d['ms_per_step'], d['step_ms_p50'], d['loss'])"
  done
done
