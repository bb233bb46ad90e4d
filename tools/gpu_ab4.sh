# A/B/C/D of env knobs on the SDXL bench in one GPU call, interleaved.  usage: bash tools/gpu_ab4.sh <tag> "<env1>" "<env2>" ... (rounds=2)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for r in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 15 --warmup 4 > gpurun_out/ab_${TAG}_${i}_$r.json 2> gpurun_out/ab_${TAG}_${i}_$r.err || { echo "bench $E failed"; tail -20 gpurun_out/ab_${TAG}_${i}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_${i}_$r.json')); print('$E', d['value'], d['ms_per_step'], d['step_ms_p50'])"
  done
done
