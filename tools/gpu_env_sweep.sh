# Same-box sweep of one env knob on the SDXL bench line (interleaved rounds).
# usage: bash tools/gpu_env_sweep.sh <tag> <VAR> <value>...  (value "-" = unset)
set -o pipefail
TAG=$1; VAR=$2; shift 2
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = "-" ]; then E=""; else E="$VAR=$v"; fi
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 15 --warmup 4 > gpurun_out/${TAG}_${v}_$r.json 2> gpurun_out/${TAG}_${v}_$r.err || { tail -20 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_${v}_$r.json')); print('$VAR=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])" | tee -a gpurun_out/${TAG}_sweep.txt
  done
done
