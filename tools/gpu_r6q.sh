# Round 6: C4 with the overlapped-norm checks on (OTAMD_NORM_CHECK=1): bookkeeping, and every overlapped chunk sum
# against the same pass over the final gradients; repeated runs.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2 3 4 5 6; do
  OTAMD_NORM_CHECK=1 timeout -k 10 200 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae --steps 4 --warmup 2 > gpurun_out/r6q.json 2> gpurun_out/r6q.err || { tail -5 gpurun_out/r6q.err; exit 1; }
  grep "norm check" gpurun_out/r6q.err | head -5
  python -c "import json; d=json.load(open('gpurun_out/r6q.json')); print('rep $rep', ' '.join(repr(v) for v in d['losses_exact']))"
done
