# A/B of two env settings on one bench model in one GPU call, interleaved:
#   usage: bash tools/gpu_ab_model.sh <tag> <model> "<envA>" "<envB>" [rounds]
set -o pipefail
TAG=$1; MODEL=$2; A=$3; B=$4; R=${5:-2}
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for arm in A B; do
    if [ $arm = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 300 python -u bench.py --model $MODEL --no-cpu-baseline --no-vae --steps 15 --warmup 4 > gpurun_out/ab_${TAG}_${arm}_$r.json 2> gpurun_out/ab_${TAG}_${arm}_$r.err || { echo "bench $arm failed"; tail -20 gpurun_out/ab_${TAG}_${arm}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_${arm}_$r.json')); print('$arm', '$E', d['value'], d['ms_per_step'], d.get('step_ms_p50'), d['roofline']['achieved'])"
  done
done
