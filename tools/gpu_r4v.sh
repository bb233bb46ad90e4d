# attention dK/dV and dQ: refill DMA pieces spread through the first sub-tile's S / dP chain (libotamd_spread.so, the working
# tree) vs the built library: parity under the alternate library, kernel A/B, step A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OTAMD_LIB_ALT=spread timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/r4v_tests.log 2>&1 || { tail -40 gpurun_out/r4v_tests.log; exit 1; }
OTAMD_LIB_ALT=spread timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_train_step_gpu.py >> gpurun_out/r4v_tests.log 2>&1 || { tail -40 gpurun_out/r4v_tests.log; exit 1; }
tail -2 gpurun_out/r4v_tests.log
for i in 1 2; do
  OTAMD_LIB_ALT=spread timeout -k 10 200 python -u tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r4v_attn_new_$i.jsonl || exit 1
  OTAMD_HOST=0 timeout -k 10 200 python -u tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r4v_attn_base_$i.jsonl || exit 1
done
for f in new_1 base_1 new_2 base_2; do echo "== $f"; cat gpurun_out/r4v_attn_$f.jsonl; done
for i in 1 2; do
  for v in new base; do
    case $v in new) E="OTAMD_HOST=0 OTAMD_LIB_ALT=spread";; base) E="OTAMD_HOST=0";; esac
    env $E timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-vae > gpurun_out/r4v_bench_${v}_${i}.json 2> gpurun_out/r4v_bench_${v}_${i}.err || { tail -20 gpurun_out/r4v_bench_${v}_${i}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4v_bench_${v}_${i}.json')); print('$v run $i', d['ms_per_step'], d['step_ms_p50'], d['loss'])"
  done
done
