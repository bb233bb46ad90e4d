set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_lora_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_lora.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_lora.log; exit 1; }
tail -1 gpurun_out/pytest_lora.log
for r in 1 2; do
for E in "OTAMD_LIB_ALT=head" "OTAMD_NOOP=1"; do
  env $E timeout -k 10 300 python -u bench.py --model sdxl-lora --no-cpu-baseline --steps 15 --warmup 4 > gpurun_out/lora_$r.json 2> gpurun_out/lora_$r.err || { echo "bench failed"; tail -20 gpurun_out/lora_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/lora_$r.json')); print('C4 $E', d['value'], d['ms_per_step'], d['step_ms_p50'])"
done
done
for E in "OTAMD_LIB_ALT=head" "OTAMD_NOOP=1"; do
  env $E timeout -k 10 400 python -u bench.py --model flux --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/fluxab.json 2> gpurun_out/fluxab.err || { echo "bench failed"; tail -20 gpurun_out/fluxab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/fluxab.json')); print('C5 $E', d['value'], d['ms_per_step'], d['step_ms_p50'])"
done
