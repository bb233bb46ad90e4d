# Round 6: C4 run-to-run determinism -- the last step's loss (full precision) over repeated short runs, default and with
# the weight-gradient stream off, the deferred split-K reduces off, and the LoRA fusion off.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae --steps 4 --warmup 2 > gpurun_out/r6n.json 2> gpurun_out/r6n.err || { echo "$name failed"; tail -5 gpurun_out/r6n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6n.json')); print('$name', repr(d['loss_exact']))"
}
for rep in 1 2 3 4 5 6; do
  run default
  run noside OTAMD_WGRAD_STREAM=0
  run nodefer OTAMD_DEFER_REDUCE=0
done
