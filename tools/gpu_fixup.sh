# In-launch split-K combine milestone: the GEMM bitwise tests, the deferred-reduce tests, then same-box A/B bench
# lines (OTAMD_GEMM_FIXUP_KB=0: every split-K GEMM launches its reduce) for the given models.
# usage: bash tools/gpu_fixup.sh <tag> <model>...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gemm_gpu.py tests/test_defer_reduce_gpu.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
grep -E "deferred reduces|passed|failed" gpurun_out/${TAG}_tests.log
for M in "$@"; do
  for kb in 0 256 0 256; do
    OTAMD_GEMM_FIXUP_KB=$kb timeout -k 10 400 python -u bench.py --model $M --no-cpu-baseline --no-vae > gpurun_out/${TAG}_${M}_${kb}.json 2> gpurun_out/${TAG}_${M}_${kb}.err || { tail -20 gpurun_out/${TAG}_${M}_${kb}.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_${M}_${kb}.json')); print('$M fixup_kb=$kb', d['value'], d['ms_per_step'], d.get('step_ms_p50'))" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
