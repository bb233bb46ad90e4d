# Round 6: FLUX embedders + modulation GEMMs + adaLN modulation sums on the weight-gradient stream -- FLUX GPU tests,
# then C5 with OTAMD_MOD_SIDE=1 vs 0, interleaved x2 (losses must be bit-identical)
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_flux_gpu.py tests/test_stream_hazards_gpu.py > gpurun_out/r6an_tests.txt 2>&1 || { tail -30 gpurun_out/r6an_tests.txt; exit 1; }
tail -1 gpurun_out/r6an_tests.txt
for r in 1 2; do
  for v in 1 0; do
    OTAMD_MOD_SIDE=$v timeout -k 10 500 python -u bench.py --model flux --no-cpu-baseline --no-vae > gpurun_out/r6an_${v}_$r.json 2> gpurun_out/r6an.err || { tail -20 gpurun_out/r6an.err; exit 1; }
  done
  python3 -c "
import json
a=json.load(open('gpurun_out/r6an_1_$r.json')); b=json.load(open('gpurun_out/r6an_0_$r.json'))
print('side', a['ms_per_step'], a['step_ms_p50'], 'main', b['ms_per_step'], b['step_ms_p50'], 'losses equal', a['losses_exact']==b['losses_exact'])"
done
