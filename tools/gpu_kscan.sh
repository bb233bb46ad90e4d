set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/kscan.log
for mn in "4096 1280" "16384 640" "4096 4096"; do
  set -- $mn
  for t in 256x256 256x128 128x256 v1; do
    KSCAN_M=$1 KSCAN_N=$2 OTAMD_GEMM_TILE=$t timeout -k 10 120 python -u tools/gemm_kscan.py >> gpurun_out/kscan.log 2>&1 || { echo "kscan failed"; tail -20 gpurun_out/kscan.log; exit 1; }
  done
done
grep -v amdgpu gpurun_out/kscan.log
