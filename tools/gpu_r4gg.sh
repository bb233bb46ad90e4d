# GEGLU fwd / bwd with 4 items per thread, loads first, 32-bit indices (libotamd_gg.so = working tree) against the
# built library (HEAD): parity tests on gg, then the SDXL step interleaved (both through the ctypes host path)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp OTAMD_HOST=0
OTAMD_LIB_ALT=gg timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_unet_gpu.py -k "geglu or unet" > gpurun_out/r4gg_tests.log 2>&1 || { tail -30 gpurun_out/r4gg_tests.log; exit 1; }
tail -1 gpurun_out/r4gg_tests.log
for i in 1 2; do
  for L in gg base; do
    if [ $L = base ]; then E="OTAMD_LIB_ALT="; else E="OTAMD_LIB_ALT=gg"; fi
    env $E timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-vae > gpurun_out/r4gg_${L}_$i.json 2> gpurun_out/r4gg_${L}_$i.err || { tail -20 gpurun_out/r4gg_${L}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4gg_${L}_$i.json')); print('$L run $i', d['ms_per_step'], d['step_ms_p50'], d['loss'])"
  done
done
