# Counter evidence of one config: GEMM-family HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and MFMA utilisation
# (one SQ/GRBM pass), written where bench.py reads them: profiles/pmc_traffic_<model>.json and
# gpurun_out/pmc_mfma_<model>.json.  usage: bash tools/gpu_counters.sh <model> [bench args...]
set -o pipefail
M=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_pmc.sh traffic_$M --model $M "$@" > gpurun_out/counters_$M.log 2>&1 || { echo "traffic $M failed"; tail -20 gpurun_out/counters_$M.log; exit 1; }
bash tools/gpu_mfma.sh mfma_$M --model $M "$@" >> gpurun_out/counters_$M.log 2>&1 || { echo "mfma $M failed"; tail -20 gpurun_out/counters_$M.log; exit 1; }
python3 -c "
import json
t = json.load(open('gpurun_out/pmc_traffic_$M.json'))
m = json.load(open('gpurun_out/pmc_mfma_$M.json'))
print('$M traffic', {k: t[k] for k in t if not isinstance(t[k], (dict, list))})
print('$M mfma', {k: m[k] for k in m if not isinstance(m[k], (dict, list))})
"
