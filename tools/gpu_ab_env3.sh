# Same-box A/B of an environment switch on the SDXL bench.  usage: bash tools/gpu_ab_env.sh VAR v1 v2 ...
# (a value "none" leaves VAR unset; extra bench arguments via BENCH_ARGS)
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
VAR=$1; shift
for rep in 1 2 3; do for v in "$@"; do
  tag=$(echo "$v" | tr '/' '_')
  if [ "$v" = none ]; then
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 15 $BENCH_ARGS > gpurun_out/abenv_$tag.json 2> gpurun_out/abenv_$tag.err || { echo "$v failed"; tail -5 gpurun_out/abenv_$tag.err; exit 1; }
  else
    env $VAR=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 15 $BENCH_ARGS > gpurun_out/abenv_$tag.json 2> gpurun_out/abenv_$tag.err || { echo "$v failed"; tail -5 gpurun_out/abenv_$tag.err; exit 1; }
  fi
  python -c "import json; d=json.load(open('gpurun_out/abenv_$tag.json')); print('$VAR=$v', d['value'], d['ms_per_step'], d['step_ms_p50'])"
done; done
