# Round 6: same-box A/B of the whole tree against the r6c tree (ab_base/: 205e5c9's package and bench.py, built):
# C5 and C3, interleaved x2
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  for M in flux sdxl; do
    timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae > gpurun_out/r6am_${M}_head_$r.json 2> gpurun_out/r6am.err || { tail -20 gpurun_out/r6am.err; exit 1; }
    (cd ab_base && timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae > ../gpurun_out/r6am_${M}_base_$r.json 2> ../gpurun_out/r6am.err) || { tail -20 gpurun_out/r6am.err; exit 1; }
    python3 -c "
import json
a=json.load(open('gpurun_out/r6am_${M}_head_$r.json')); b=json.load(open('gpurun_out/r6am_${M}_base_$r.json'))
print('$M head', a['ms_per_step'], a['step_ms_p50'], 'r6c', b['ms_per_step'], b['step_ms_p50'])"
  done
done
