# Round 6: fused-LoRA tile sweep at the aspect buckets' row counts (level 2 / level 1: 4032 / 16128, 4160 / 16640)
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for ms in 4032,16128 4160,16640; do
  timeout -k 10 300 python -u tools/lora_ld_tile_sweep.py --ms $ms >> gpurun_out/r6_lora_ld_tiles_arb.jsonl 2> gpurun_out/r6ao.err || { tail -5 gpurun_out/r6ao.err; exit 1; }
done
cat gpurun_out/r6_lora_ld_tiles_arb.jsonl
