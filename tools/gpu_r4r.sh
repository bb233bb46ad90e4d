# cross-attention dK/dV chunk sum on the weight-gradient stream + clamped-exp padded keys in the cross kernel:
# parity, step tests, kernel A/B against HEAD, step A/B (new / cast on main / HEAD)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/r4r_tests_attn.log 2>&1 || { tail -40 gpurun_out/r4r_tests_attn.log; exit 1; }
tail -2 gpurun_out/r4r_tests_attn.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_train_step_gpu.py tests/test_host_layer_gpu.py tests/test_lora_gpu.py "tests/test_fullsize_gpu.py::test_full_unet_matches_oracle[sdxl-512]" > gpurun_out/r4r_tests.log 2>&1 || { tail -40 gpurun_out/r4r_tests.log; exit 1; }
tail -2 gpurun_out/r4r_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r4r_attn_new_$i.jsonl || exit 1
  OTAMD_LIB_ALT=base timeout -k 10 200 python -u tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r4r_attn_base_$i.jsonl || exit 1
done
for f in new_1 base_1 new_2 base_2; do echo "== $f"; cat gpurun_out/r4r_attn_$f.jsonl; done
for i in 1 2; do
  for v in new castmain base; do
    case $v in new) E="OTAMD_HOST=0";; castmain) E="OTAMD_HOST=0 OTAMD_CROSS_CAST_SIDE=0";; base) E="OTAMD_HOST=0 OTAMD_LIB_ALT=base OTAMD_CROSS_CAST_SIDE=0";; esac
    env $E timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-vae > gpurun_out/r4r_bench_${v}_${i}.json 2> gpurun_out/r4r_bench_${v}_${i}.err || { tail -20 gpurun_out/r4r_bench_${v}_${i}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4r_bench_${v}_${i}.json')); print('$v run $i', d['ms_per_step'], d['step_ms_p50'], d['loss'])"
  done
done
