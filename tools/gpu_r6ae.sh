# Round 6: weight-gradient-only LoRA backward (and the LoRA cross-attention dK/dV sum) on the side stream --
# LoRA / hazard / step GPU tests, the full-width SDXL LoRA oracle test, then C4 / C5 with OTAMD_WGRAD_ONLY_SIDE=1 vs 0
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_stream_hazards_gpu.py tests/test_lora_gpu.py tests/test_defer_reduce_gpu.py tests/test_train_step_gpu.py "tests/test_fullsize_gpu.py::test_full_width_sdxl_lora_r32_matches_oracle" > gpurun_out/r6ae_tests.txt 2>&1 || { tail -30 gpurun_out/r6ae_tests.txt; exit 1; }
tail -1 gpurun_out/r6ae_tests.txt
for r in 1 2; do
  for M in sdxl-lora flux; do
    for v in 1 0; do
      OTAMD_WGRAD_ONLY_SIDE=$v timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae > gpurun_out/r6ae_${M}_${v}_$r.json 2> gpurun_out/r6ae.err || { tail -20 gpurun_out/r6ae.err; exit 1; }
    done
    python3 -c "
import json
a=json.load(open('gpurun_out/r6ae_${M}_1_$r.json')); b=json.load(open('gpurun_out/r6ae_${M}_0_$r.json'))
print('$M', 'side', a['ms_per_step'], a['step_ms_p50'], 'main', b['ms_per_step'], b['step_ms_p50'], 'losses equal', a['losses_exact']==b['losses_exact'])"
  done
done
