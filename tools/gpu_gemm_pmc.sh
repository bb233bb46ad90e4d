# PMC passes over one GEMM shape (tools/gemm_one.py).  usage: bash tools/gpu_gemm_pmc.sh <tag> <gemm_one args...>
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_${TAG}_$i
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_$i -o run -- python3 -u tools/gemm_one.py "$@" --reps 20 > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -20 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
  python3 tools/pmc_kernels.py gpurun_out/pmc_${TAG}_$i | grep -E "gemm2|splitk" > gpurun_out/pmc_${TAG}_$i.txt
  cat gpurun_out/pmc_${TAG}_$i.txt
  rm -rf gpurun_out/pmc_${TAG}_$i
done
