# dK/dV bias records (lse / delta folded into the MFMA chains): parity + kernel A/B against libotamd_base.so
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py::test_attention tests/test_host_layer_gpu.py tests/test_train_step_gpu.py tests/test_flux_gpu.py > gpurun_out/r4h_tests.log 2>&1 || { tail -40 gpurun_out/r4h_tests.log; exit 1; }
tail -3 gpurun_out/r4h_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r4h_attn_new_$i.jsonl || exit 1
  OTAMD_LIB_ALT=base timeout -k 10 200 python -u tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu.ids > gpurun_out/r4h_attn_base_$i.jsonl || exit 1
done
for f in new_1 base_1 new_2 base_2; do echo "== $f"; cat gpurun_out/r4h_attn_$f.jsonl; done
rm -rf gpurun_out/kp_r4g
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kp_r4g -o run -- python3 -u tools/attn_bench.py --reps 10 > gpurun_out/kp_r4g.log 2>&1 || { tail -20 gpurun_out/kp_r4g.log; exit 1; }
python3 tools/ktrace_by_grid.py gpurun_out/kp_r4g --match attn --top 40 | tee gpurun_out/r4g_attn_by_grid.txt
rm -rf gpurun_out/kp_r4g
