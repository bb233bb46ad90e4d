# round 4: one-pass cross-attention backward + XCD-grouped attention block order -- parity, determinism, kernel timings,
# same-box step A/B (OTAMD_ATTN_CROSS_OFF=1 OTAMD_ATTN_XCD=0 = the round-3 attention)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py::test_attention tests/test_train_step_gpu.py::test_full_sdxl_steps_bitwise_repeatable > gpurun_out/r4b_tests.log 2>&1 || { tail -40 gpurun_out/r4b_tests.log; exit 1; }
tail -3 gpurun_out/r4b_tests.log
timeout -k 10 200 python -u tools/attn_bench.py --reps 20 > gpurun_out/r4b_attn_new.jsonl 2>&1 || exit 1
OTAMD_ATTN_CROSS_OFF=1 OTAMD_ATTN_XCD=0 timeout -k 10 200 python -u tools/attn_bench.py --reps 20 > gpurun_out/r4b_attn_old.jsonl 2>&1 || exit 1
for f in new old; do echo "== $f"; grep -v amdgpu.ids gpurun_out/r4b_attn_$f.jsonl; done
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export OTAMD_ATTN_CROSS_OFF=1 OTAMD_ATTN_XCD=0; else unset OTAMD_ATTN_CROSS_OFF OTAMD_ATTN_XCD; fi
    timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-vae > gpurun_out/r4b_bench_${v}_${i}.json 2> gpurun_out/r4b_bench_${v}_${i}.err || { tail -20 gpurun_out/r4b_bench_${v}_${i}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4b_bench_${v}_${i}.json')); print('$v run $i', d['ms_per_step'], d['step_ms_p50'], d['loss'])"
  done
done
