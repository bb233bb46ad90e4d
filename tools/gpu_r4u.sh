# GEMM: s_setprio(1) around the MFMA phases (T5) vs HEAD: parity, shape A/B, step A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_gpu.py tests/test_train_step_gpu.py tests/test_host_layer_gpu.py > gpurun_out/r4u_tests.log 2>&1 || { tail -40 gpurun_out/r4u_tests.log; exit 1; }
tail -2 gpurun_out/r4u_tests.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r4u_gemm_new_$i.jsonl || exit 1
  OTAMD_LIB_ALT=base timeout -k 10 300 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r4u_gemm_base_$i.jsonl || exit 1
done
python3 - <<'PY'
import json
def load(f): return {r['name']: r for r in map(json.loads, open(f))}
for i in (1, 2):
    n, b = load(f'gpurun_out/r4u_gemm_new_{i}.jsonl'), load(f'gpurun_out/r4u_gemm_base_{i}.jsonl')
    for k in n:
        print(i, k, *[f"{op} {n[k][op]:.0f}/{b[k][op]:.0f}" for op in ('fwd', 'dgrad', 'wgrad')])
PY
for i in 1 2; do
  for v in new base; do
    case $v in new) E="OTAMD_HOST=0";; base) E="OTAMD_HOST=0 OTAMD_LIB_ALT=base";; esac
    env $E timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-vae > gpurun_out/r4u_bench_${v}_${i}.json 2> gpurun_out/r4u_bench_${v}_${i}.err || { tail -20 gpurun_out/r4u_bench_${v}_${i}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4u_bench_${v}_${i}.json')); print('$v run $i', d['ms_per_step'], d['step_ms_p50'], d['loss'])"
  done
done
