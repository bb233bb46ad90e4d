# Whole-step HIP graph (OTAMD_STEP_GRAPH=1) re-measured against the eager two-stream step, with the HIP runtime's
# graph execution knobs (DEBUG_HIP_FORCE_GRAPH_QUEUES: streams for parallel graph branches; packet capture), and its
# host issue time
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 --no-cpu-baseline --no-vae > gpurun_out/r4z_$name.json 2> gpurun_out/r4z_$name.err || { tail -20 gpurun_out/r4z_$name.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4z_$name.json')); print('$name', d['ms_per_step'], d['step_ms_p50'], d['loss'], d.get('step_graph', '')[:40])"
}
run eager OTAMD_STEP_GRAPH=0 &&
run graph OTAMD_STEP_GRAPH=1 &&
run graph_q1 OTAMD_STEP_GRAPH=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1 &&
run graph_q2 OTAMD_STEP_GRAPH=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 &&
run graph_q8 OTAMD_STEP_GRAPH=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=8 &&
run graph_nopc OTAMD_STEP_GRAPH=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 &&
OTAMD_STEP_GRAPH=1 timeout -k 10 300 python -u tools/host_overhead.py > gpurun_out/r4z_host_graph.txt 2>&1 && grep step gpurun_out/r4z_host_graph.txt
