# Same-box A/B of an environment switch on the SDXL bench.  usage: bash tools/gpu_ab_env.sh VAR v1 v2 ...
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
VAR=$1; shift
for rep in 1 2; do for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 15 > gpurun_out/abenv_$v.json 2> gpurun_out/abenv_$v.err || { echo "$v failed"; tail -5 gpurun_out/abenv_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/abenv_$v.json')); print('$VAR=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
done; done
