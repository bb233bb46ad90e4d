# Round 6: spread refills in the LoRA second-segment GEMMs -- tests, then C5 / C4 with the HEAD library against the
# working tree's (both through OTAMD_LIB_ALT, i.e. the ctypes host path in both arms), interleaved x2.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_lora_fused_gpu.py tests/test_lora_gpu.py tests/test_gemm_gpu.py tests/test_flux_gpu.py > gpurun_out/r6l_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6l_tests.log; grep -E "FAILED|Error" gpurun_out/r6l_tests.log | head -10
[ $rc -ne 0 ] && exit 1
run() {  # model, name, env...
  local m=$1 name=$2; shift 2
  env "$@" timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline --no-vae --steps 12 > gpurun_out/r6l_${m}_$name.json 2> gpurun_out/r6l_${m}_$name.err || { echo "$m $name failed"; tail -5 gpurun_out/r6l_${m}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6l_${m}_$name.json')); print('$m $name', d['value'], d['ms_per_step'], d['step_ms_p50'], d['loss'])"
}
for rep in 1 2; do
  for m in flux sdxl-lora; do
    run $m head OTAMD_LIB_ALT=head
    run $m new OTAMD_LIB_ALT=new
  done
done
