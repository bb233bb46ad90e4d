# A/B of the step graph and the weight-gradient side stream (SDXL 1024^2 b=4).  usage: bash tools/gpu_graph_ab.sh <tag>
set -o pipefail
TAG=${1:-ab}
export TMPDIR=/tmp
mkdir -p gpurun_out
for G in 1 0; do for S in 1 0; do
  OTAMD_STEP_GRAPH=$G OTAMD_WGRAD_STREAM=$S timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 10 --warmup 3 > gpurun_out/ab_${TAG}_g${G}s${S}.json 2> gpurun_out/ab_${TAG}_g${G}s${S}.err || { echo "bench failed g$G s$S"; tail -20 gpurun_out/ab_${TAG}_g${G}s${S}.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_g${G}s${S}.json')); print('graph $G stream $S', d['value'], d['step_ms_p50'])"
done; done
