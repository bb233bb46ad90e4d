# Same-box A/B: AdamW on its own stream beside the next forward (OTAMD_OPT_OVERLAP=1) with its grid capped
# (OTAMD_ADAMW_BLOCKS), against the in-line update.  usage: bash tools/gpu_ab_optoverlap.sh <tag> caps...
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=$1; shift
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 15 > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { echo "$name failed"; tail -5 gpurun_out/${TAG}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_$name.json')); print('$name', d['value'], d['ms_per_step'], d['step_ms_p50'], d['loss'])"
}
for rep in 1 2; do
  run base OTAMD_OPT_OVERLAP=0
  for c in "$@"; do run ov$c OTAMD_OPT_OVERLAP=1 OTAMD_ADAMW_BLOCKS=$c; done
done
