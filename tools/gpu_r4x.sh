# D = 128 (FLUX) attention backward variants as alternate libraries: f1 = dK/dV 32-query stages, f2 = dQ 64-key
# tiles 2-deep, against cur (the same tree otherwise): parity on the D = 128 shapes, kernel A/B, C5 step A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp OTAMD_HOST=0
for L in f1 f2; do
  OTAMD_LIB_ALT=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention and 128" > gpurun_out/r4x_tests_$L.log 2>&1 || { tail -30 gpurun_out/r4x_tests_$L.log; exit 1; }
  tail -1 gpurun_out/r4x_tests_$L.log
done
for i in 1 2; do
  for L in cur f1 f2; do
    OTAMD_LIB_ALT=$L timeout -k 10 200 python -u tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu.ids | grep "128\]" > gpurun_out/r4x_attn_${L}_$i.jsonl || exit 1
    echo "$L $i $(cat gpurun_out/r4x_attn_${L}_$i.jsonl)"
  done
done
for L in cur f1 f2; do
  OTAMD_LIB_ALT=$L timeout -k 10 400 python -u bench.py --model flux --steps 6 --warmup 2 --no-cpu-baseline --no-vae > gpurun_out/r4x_flux_$L.json 2> gpurun_out/r4x_flux_$L.err || { tail -20 gpurun_out/r4x_flux_$L.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4x_flux_$L.json')); print('flux $L', d['ms_per_step'], d['step_ms_p50'], d['loss'])"
done
