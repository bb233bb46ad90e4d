set -o pipefail
mkdir -p gpurun_out
for t in 4 7 0; do
  KSCAN_M=4096 KSCAN_N=1280 OTAMD_GEMM_TABLE=0 OTAMD_GEMM_TILE=$t timeout -k 10 120 python3 -u tools/gemm_kscan.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r4k_kscan.jsonl
done
KSCAN_M=4096 KSCAN_N=4096 OTAMD_GEMM_TABLE=0 OTAMD_GEMM_TILE=0 timeout -k 10 120 python3 -u tools/gemm_kscan.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r4k_kscan.jsonl
