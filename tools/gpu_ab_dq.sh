# A/B on one box: dQ ring depth 2 (default, 3 blocks/CU) vs 3.  usage: bash tools/gpu_ab_dq.sh <tag>
set -o pipefail
TAG=${1:-dq}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for V in 0 1; do
  rm -rf gpurun_out/prof_${TAG}_$V
  OTAMD_ATTN_DQ_NS3=$V timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_${TAG}_$V -o run -- python3 -u bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-vae > gpurun_out/prof_${TAG}_$V.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_${TAG}_$V.log; exit 1; }
done
for R in 1 2; do for V in 0 1; do
  OTAMD_ATTN_DQ_NS3=$V timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 20 --warmup 4 > gpurun_out/ab_${TAG}_${R}_${V}.json 2>/dev/null || { echo "bench failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_${R}_${V}.json')); print('run $R ns3 $V', d['value'], d['step_ms_p50'])"
done; done
