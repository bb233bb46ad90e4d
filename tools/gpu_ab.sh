# A/B of an env knob on the SDXL bench in one GPU call, interleaved: usage: bash tools/gpu_ab.sh <tag> "<envA>" "<envB>" [rounds]
set -o pipefail
TAG=$1; A=$2; B=$3; R=${4:-2}
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for arm in A B; do
    if [ $arm = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 15 --warmup 4 > gpurun_out/ab_${TAG}_${arm}_$r.json 2> gpurun_out/ab_${TAG}_${arm}_$r.err || { echo "bench $arm failed"; tail -20 gpurun_out/ab_${TAG}_${arm}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_${arm}_$r.json')); print('$arm', '$E', d['value'], d['ms_per_step'], d['step_ms_p50'], d['roofline']['achieved'])"
  done
done
