# GEMM parity for every forced v2 tile, then the microbenchmark (default plan and 4-wave 256x256)
set -o pipefail
mkdir -p gpurun_out
for t in 256x256 256x128 128x256 256x256w4; do
  OTAMD_GEMM_TILE=$t timeout -k 10 300 python -m pytest tests/test_gemm_gpu.py -q -x > gpurun_out/v2_$t.log 2>&1 || { echo "FAIL $t" >> gpurun_out/v2_summary.log; exit 1; }
  echo "ok $t $(tail -1 gpurun_out/v2_$t.log)" >> gpurun_out/v2_summary.log
done
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm2.log 2>&1
OTAMD_GEMM_TILE=256x256w4 timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm2_w4.log 2>&1
