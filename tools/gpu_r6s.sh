# Round 6: C4 run-to-run determinism with the skinny tiles (5 / 6) on their 4-deep-ring variants (OTAMD_SKINNY_NS4=1)
# against the default, 12 runs each, interleaved; first timed-step loss in full precision.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae --steps 2 --warmup 2 > gpurun_out/r6s.json 2> gpurun_out/r6s.err || { echo "$name failed"; tail -5 gpurun_out/r6s.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6s.json')); print('$name', ' '.join(repr(v) for v in d['losses_exact']))"
}
for rep in $(seq 1 12); do
  run default
  run ns4 OTAMD_SKINNY_NS4=1
done
