# Same-box sweep of the in-launch split-K combine's per-tile byte limit (OTAMD_GEMM_FIXUP_KB) on bench lines.
# usage: bash tools/gpu_fixup_sweep.sh <tag> <model> <kb>...
set -o pipefail
TAG=$1; M=$2; shift 2
mkdir -p gpurun_out
for rep in 1 2; do
  for kb in "$@"; do
    OTAMD_GEMM_FIXUP_KB=$kb timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae > gpurun_out/${TAG}_${M}_${kb}.json 2> gpurun_out/${TAG}_${M}_${kb}.err || { tail -20 gpurun_out/${TAG}_${M}_${kb}.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_${M}_${kb}.json')); print('$M fixup_kb=$kb', d['value'], d['ms_per_step'], d.get('step_ms_p50'))" | tee -a gpurun_out/${TAG}_sweep.txt
  done
done
