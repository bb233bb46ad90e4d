# Same-box A/B of the whole-step HIP graph (OTAMD_STEP_GRAPH=1) against the eager two-stream step, with the
# HIP runtime's graph execution modes: packet capture (the default: the graph's AQL packets recorded and
# submitted as one batch on one queue) vs per-node submission over several queues.  usage: bash tools/gpu_ab_graph.sh
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
run() {   # tag, env assignments...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 15 > gpurun_out/abg_$tag.json 2> gpurun_out/abg_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/abg_$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/abg_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['step_ms_p50'])"
}
for rep in 1 2; do
  run eager OTAMD_STEP_GRAPH=0 || exit 1
  run graph OTAMD_STEP_GRAPH=1 || exit 1
  run graph_nopc OTAMD_STEP_GRAPH=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
  run graph_nopc_q4 OTAMD_STEP_GRAPH=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 || exit 1
done
