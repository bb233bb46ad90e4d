# Round 6: measured fused-LoRA tile choices (lora_plans_mi355x.json) -- fused-LoRA GPU tests, then C4 with
# OTAMD_LORA_PLANS=1 vs 0, 3 interleaved rounds
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_lora_fused_gpu.py "tests/test_fullsize_gpu.py::test_full_width_sdxl_lora_r32_matches_oracle" > gpurun_out/r6ah_tests.txt 2>&1 || { tail -30 gpurun_out/r6ah_tests.txt; exit 1; }
tail -1 gpurun_out/r6ah_tests.txt
for r in 1 2 3; do
  for v in 1 0; do
    OTAMD_LORA_PLANS=$v timeout -k 10 400 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae > gpurun_out/r6ah_${v}_$r.json 2> gpurun_out/r6ah.err || { tail -20 gpurun_out/r6ah.err; exit 1; }
  done
  python3 -c "
import json
a=json.load(open('gpurun_out/r6ah_1_$r.json')); b=json.load(open('gpurun_out/r6ah_0_$r.json'))
print('table', a['ms_per_step'], a['step_ms_p50'], 'plan-tile', b['ms_per_step'], b['step_ms_p50'], a['lora_forwards_fused_vs_two_launch'], b['lora_forwards_fused_vs_two_launch'])"
done
