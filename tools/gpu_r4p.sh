# last-tile-only key masking in the attention forward / dQ kernels: parity, kernel A/B against HEAD, step A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/r4p_tests_attn.log 2>&1 || { tail -40 gpurun_out/r4p_tests_attn.log; exit 1; }
tail -2 gpurun_out/r4p_tests_attn.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_train_step_gpu.py tests/test_flux_gpu.py > gpurun_out/r4p_tests.log 2>&1 || { tail -40 gpurun_out/r4p_tests.log; exit 1; }
tail -2 gpurun_out/r4p_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r4p_attn_new_$i.jsonl || exit 1
  OTAMD_LIB_ALT=base timeout -k 10 200 python -u tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r4p_attn_base_$i.jsonl || exit 1
done
for f in new_1 base_1 new_2 base_2; do echo "== $f"; cat gpurun_out/r4p_attn_$f.jsonl; done
for i in 1 2; do
  for v in new base; do
    case $v in new) E="OTAMD_HOST=0";; base) E="OTAMD_HOST=0 OTAMD_LIB_ALT=base";; esac
    env $E timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-vae > gpurun_out/r4p_bench_${v}_${i}.json 2> gpurun_out/r4p_bench_${v}_${i}.err || { tail -20 gpurun_out/r4p_bench_${v}_${i}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4p_bench_${v}_${i}.json')); print('$v run $i', d['ms_per_step'], d['step_ms_p50'], d['loss'])"
  done
done
bash tools/gpu_r4o.sh
