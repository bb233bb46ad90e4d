# FLUX milestone: the Flux tests (full-width blocks vs the oracle, LoRA steps), then a same-box A/B of the C5 bench
# line over an env knob.   usage: bash tools/gpu_flux_ab.sh <tag> <VAR>   (arms VAR=0 / VAR=1)
set -o pipefail
TAG=$1; VAR=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_flux_gpu.py "tests/test_fullsize_gpu.py::test_full_width_flux_blocks_768_match_oracle" "tests/test_fullsize_gpu.py::test_flux_lora_768_b4" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for v in 0 1 0 1; do
  env $VAR=$v timeout -k 10 400 python -u bench.py --model flux --no-cpu-baseline --no-vae > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || { tail -20 gpurun_out/${TAG}_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$v.json')); print('flux $VAR=$v', d['value'], d['ms_per_step'], d.get('step_ms_p50'))" | tee -a gpurun_out/${TAG}_ab.txt
done
