# Round 6: C4 determinism hunt -- per-step adapter-gradient digests over 5 runs (tools/lora_grad_digest.py), then the
# skinny tiles on their 4-deep-ring variants (OTAMD_SKINNY_NS4=1) against the default, 10 runs each.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2 3 4 5; do
  timeout -k 10 200 python -u tools/lora_grad_digest.py --steps 3 > gpurun_out/r6s_digest_$rep.txt 2> gpurun_out/r6s_digest.err || { tail -5 gpurun_out/r6s_digest.err; exit 1; }
  grep "^step" gpurun_out/r6s_digest_$rep.txt
done
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae --steps 2 --warmup 2 > gpurun_out/r6s.json 2> gpurun_out/r6s.err || { echo "$name failed"; tail -5 gpurun_out/r6s.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6s.json')); print('$name', ' '.join(repr(v) for v in d['losses_exact']))"
}
for rep in $(seq 1 10); do
  run default
  run ns4 OTAMD_SKINNY_NS4=1
done
