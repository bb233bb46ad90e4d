# Round 6: LoRA backward input gradient with u = dy (sB) fused into the dgrad GEMM (single-module and q|k|v sites) -- fused-LoRA GPU tests, LoRA /
# hazard tests, the full-width SDXL LoRA oracle test, then C4 with OTAMD_LORA_FUSE_DGRAD=1 vs 0 interleaved
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_lora_fused_gpu.py tests/test_lora_gpu.py tests/test_stream_hazards_gpu.py "tests/test_fullsize_gpu.py::test_full_width_sdxl_lora_r32_matches_oracle" > gpurun_out/r6af_tests.txt 2>&1 || { tail -30 gpurun_out/r6af_tests.txt; exit 1; }
tail -1 gpurun_out/r6af_tests.txt
for r in 1 2; do
  for v in 1 0; do
    OTAMD_LORA_FUSE_DGRAD=$v timeout -k 10 400 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae > gpurun_out/r6af_${v}_$r.json 2> gpurun_out/r6af.err || { tail -20 gpurun_out/r6af.err; exit 1; }
  done
  python3 -c "
import json
a=json.load(open('gpurun_out/r6af_1_$r.json')); b=json.load(open('gpurun_out/r6af_0_$r.json'))
print('fused', a['ms_per_step'], a['step_ms_p50'], 'two-launch', b['ms_per_step'], b['step_ms_p50'], 'losses equal', a['losses_exact']==b['losses_exact'])"
done
