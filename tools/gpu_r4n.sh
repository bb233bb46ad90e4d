# dual-use attention LDS images (one Q / dO / K copy for row and transposed reads; 64-query dK/dV stages):
# parity, kernel A/B against HEAD's library, step A/B (+ the opt-in overlapped AdamW); attention per-grid kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/r4n_tests_attn.log 2>&1 || { tail -40 gpurun_out/r4n_tests_attn.log; exit 1; }
tail -2 gpurun_out/r4n_tests_attn.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_host_layer_gpu.py tests/test_train_step_gpu.py tests/test_flux_gpu.py tests/test_lora_gpu.py \
  "tests/test_fullsize_gpu.py::test_full_unet_matches_oracle[sdxl-512]" > gpurun_out/r4n_tests.log 2>&1 || { tail -40 gpurun_out/r4n_tests.log; exit 1; }
tail -2 gpurun_out/r4n_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r4n_attn_new_$i.jsonl || exit 1
  OTAMD_LIB_ALT=base timeout -k 10 200 python -u tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r4n_attn_base_$i.jsonl || exit 1
done
for f in new_1 base_1 new_2 base_2; do echo "== $f"; cat gpurun_out/r4n_attn_$f.jsonl; done
for i in 1 2; do
  for v in new base ovl; do
    case $v in new) E="OTAMD_HOST=0";; base) E="OTAMD_HOST=0 OTAMD_LIB_ALT=base";; ovl) E="OTAMD_HOST=0 OTAMD_OPT_OVERLAP=1";; esac
    env $E timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-vae > gpurun_out/r4n_bench_${v}_${i}.json 2> gpurun_out/r4n_bench_${v}_${i}.err || { tail -20 gpurun_out/r4n_bench_${v}_${i}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4n_bench_${v}_${i}.json')); print('$v run $i', d['ms_per_step'], d['step_ms_p50'], d['loss'])"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4n_attn -o attn -- python3 $GRAFT_REPO_ROOT/tools/attn_bench.py --reps 5 > $GRAFT_REPO_ROOT/gpurun_out/r4n_attn.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4n_attn.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/ktrace_by_grid.py gpurun_out/r4n_attn --match attn > gpurun_out/r4n_attn_grid.txt && cat gpurun_out/r4n_attn_grid.txt
