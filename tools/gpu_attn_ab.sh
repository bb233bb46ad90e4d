set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/attn_t.log 2>&1; rc=$?; tail -3 gpurun_out/attn_t.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  OTAMD_HOST=0 timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_new_$r.jsonl || exit 1
  OTAMD_LIB_ALT=base timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_base_$r.jsonl || exit 1
done
