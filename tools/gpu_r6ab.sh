# Round 6: time-embedding branch on the weight-gradient stream -- hazard / step GPU tests, then C3 / C4 / C2 steps
# with OTAMD_TEMB_SIDE=1 vs 0 interleaved on one box (losses must be bit-identical)
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_stream_hazards_gpu.py tests/test_train_step_gpu.py > gpurun_out/r6ab_tests.txt 2>&1 || { tail -30 gpurun_out/r6ab_tests.txt; exit 1; }
tail -1 gpurun_out/r6ab_tests.txt
for r in 1 2; do
  for M in sdxl sdxl-lora sd15; do
    for v in 1 0; do
      OTAMD_TEMB_SIDE=$v timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae > gpurun_out/r6ab_${M}_${v}_$r.json 2> gpurun_out/r6ab.err || { tail -20 gpurun_out/r6ab.err; exit 1; }
    done
    python3 -c "
import json,sys
a=json.load(open('gpurun_out/r6ab_${M}_1_$r.json')); b=json.load(open('gpurun_out/r6ab_${M}_0_$r.json'))
print('$M', 'side', a['ms_per_step'], a['step_ms_p50'], 'main', b['ms_per_step'], b['step_ms_p50'], 'losses equal', a['losses_exact']==b['losses_exact'])"
  done
done
