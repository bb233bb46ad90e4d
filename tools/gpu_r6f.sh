# Round 6: fused LoRA down-projection -- its kernel tests, the LoRA / host-layer / defer suites, the full-width SDXL LoRA
# oracle test, then C4 with the fusion on and off (interleaved x2).
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_lora_fused_gpu.py > gpurun_out/r6f_fused.log 2>&1; rc=$?
tail -3 gpurun_out/r6f_fused.log; grep -E "FAILED|Error" gpurun_out/r6f_fused.log | head -10
[ $rc -ne 0 ] && exit 1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_lora_gpu.py tests/test_host_layer_gpu.py tests/test_defer_reduce_gpu.py tests/test_gemm_gpu.py "tests/test_fullsize_gpu.py::test_full_width_sdxl_lora_r32_matches_oracle" "tests/test_fullsize_gpu.py::test_sdxl_lora_r32_aspect_buckets" > gpurun_out/r6f_suite.log 2>&1; rc=$?
tail -3 gpurun_out/r6f_suite.log; grep -E "FAILED|Error" gpurun_out/r6f_suite.log | head -10
[ $rc -ne 0 ] && exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae --steps 15 > gpurun_out/r6f_$name.json 2> gpurun_out/r6f_$name.err || { echo "$name failed"; tail -5 gpurun_out/r6f_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6f_$name.json')); print('$name', d['value'], d['ms_per_step'], d['step_ms_p50'], d['loss'])"
}
for rep in 1 2; do
  run fuse0 OTAMD_LORA_FUSE=0
  run fuse1 OTAMD_LORA_FUSE=1
done
