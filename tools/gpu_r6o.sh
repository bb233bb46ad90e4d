# Round 6: C4 run-to-run determinism by component: default, clip norm not overlapped (OTAMD_NORM_OVERLAP=0), side
# stream off; the per-step losses in full precision.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae --steps 5 --warmup 2 > gpurun_out/r6o.json 2> gpurun_out/r6o.err || { echo "$name failed"; tail -5 gpurun_out/r6o.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6o.json')); print('$name', ' '.join(repr(v) for v in d['losses_exact']))"
}
for rep in 1 2 3 4 5 6 7 8 9 10; do
  run default
  run nonorm OTAMD_NORM_OVERLAP=0

done
