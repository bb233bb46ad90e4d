# dgrad issued before the weight-gradient region (fork point recorded first) vs HEAD's order (ab_old/ = HEAD's
# tree): step-graph / eager parity tests, then eager and whole-step-graph benches interleaved, plus the graph's
# host issue time
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_train_step_gpu.py tests/test_host_layer_gpu.py > gpurun_out/r4fork_tests.log 2>&1 || { tail -40 gpurun_out/r4fork_tests.log; exit 1; }
tail -1 gpurun_out/r4fork_tests.log
run() {   # name, dir, env...
  local name=$1 dir=$2; shift 2
  (cd $dir && env "$@" timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 --no-cpu-baseline --no-vae) > gpurun_out/r4fork_$name.json 2> gpurun_out/r4fork_$name.err || { tail -20 gpurun_out/r4fork_$name.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4fork_$name.json')); print('$name', d['ms_per_step'], d['step_ms_p50'], d['loss'])"
}
for i in 1 2; do
  run eager_new_$i . OTAMD_STEP_GRAPH=0 && run eager_old_$i ab_old OTAMD_STEP_GRAPH=0 &&
  run graph_new_$i . OTAMD_STEP_GRAPH=1 && run graph_old_$i ab_old OTAMD_STEP_GRAPH=1 || exit 1
done
run graph_new_q2 . OTAMD_STEP_GRAPH=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 &&
OTAMD_STEP_GRAPH=1 timeout -k 10 300 python -u tools/host_overhead.py > gpurun_out/r4fork_host_graph.txt 2>&1 && grep step gpurun_out/r4fork_host_graph.txt
