# LayerNorm parameter reduction + time-embedding subgraph on the weight-gradient stream: parity + step A/B; GEMM K-scan
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "layernorm" tests/test_host_layer_gpu.py tests/test_train_step_gpu.py tests/test_lora_gpu.py \
  tests/test_dp_gpu.py tests/test_backup_gpu.py "tests/test_fullsize_gpu.py::test_full_unet_matches_oracle[sdxl-512]" > gpurun_out/r4l_tests.log 2>&1 || { tail -40 gpurun_out/r4l_tests.log; exit 1; }
tail -3 gpurun_out/r4l_tests.log
for i in 1 2; do
  for v in on lnoff tembof; do
    case $v in on) E="OTAMD_LN_REDUCE_SIDE=1";; lnoff) E="OTAMD_LN_REDUCE_SIDE=0";; tembof) E="OTAMD_TEMB_SIDE=0";; esac
    env $E timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-vae > gpurun_out/r4l_bench_${v}_${i}.json 2> gpurun_out/r4l_bench_${v}_${i}.err || { tail -20 gpurun_out/r4l_bench_${v}_${i}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4l_bench_${v}_${i}.json')); print('$v run $i', d['ms_per_step'], d['step_ms_p50'], d['loss'])"
  done
done
bash tools/gpu_r4k.sh
