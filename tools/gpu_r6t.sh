# Round 6: C4 determinism hunt -- per-step adapter-gradient digests over the aspect buckets, 6 runs.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2 3 4 5 6; do
  timeout -k 10 300 python -u tools/lora_grad_digest.py --steps 9 --arb > gpurun_out/r6t_digest_$rep.txt 2> gpurun_out/r6t_digest.err || { tail -5 gpurun_out/r6t_digest.err; exit 1; }
  grep "^step" gpurun_out/r6t_digest_$rep.txt | awk '{print $2, $4}' | tr '\n' ' '; echo
done
