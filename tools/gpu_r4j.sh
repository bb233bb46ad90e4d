# GEMM K-loop ablations: kernel durations per (kernel, grid) for the real kernel and ablations 1..4
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in real abl1 abl2 abl3 abl4; do
  rm -rf gpurun_out/kp_$v
  if [ $v = real ]; then E="OTAMD_HOST=0"; else E="OTAMD_LIB_ALT=$v"; fi
  env $E timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/kp_$v -o run -- python3 -u tools/gemm_abl_run.py --reps 30 > gpurun_out/kp_$v.log 2>&1 || { tail -20 gpurun_out/kp_$v.log; exit 1; }
  echo "== $v"
  python3 tools/ktrace_by_grid.py gpurun_out/kp_$v --match gemm2 --top 12 | tee gpurun_out/r4j_$v.txt
  rm -rf gpurun_out/kp_$v
done
