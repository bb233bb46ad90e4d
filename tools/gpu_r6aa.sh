# Round 6: cost of the LDS-waiting ring barriers -- attention kernels alone and C3 / C4 steps, new vs base (522c930),
# interleaved on one box
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  OTAMD_HOST=0 timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/r6aa_attn_new_$r.jsonl || exit 1
  OTAMD_HOST=0 OTAMD_LIB_ALT=base timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/r6aa_attn_base_$r.jsonl || exit 1
done
for r in 1 2; do
  for M in sdxl sdxl-lora; do
    timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae > gpurun_out/r6aa_${M}_new_$r.json 2> gpurun_out/r6aa.err || exit 1
    OTAMD_LIB_ALT=base timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae > gpurun_out/r6aa_${M}_base_$r.json 2> gpurun_out/r6aa.err || exit 1
    python -c "import json,sys; [print(f, json.load(open(f))['ms_per_step']) for f in sys.argv[1:]]" gpurun_out/r6aa_${M}_new_$r.json gpurun_out/r6aa_${M}_base_$r.json
  done
done
