# Round 6: after the attention ring barriers wait for LDS reads -- attention GPU tests, then 40 C4 determinism runs
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/r6z_attn_tests.txt 2>&1 || { tail -20 gpurun_out/r6z_attn_tests.txt; exit 1; }
tail -2 gpurun_out/r6z_attn_tests.txt
bash tools/gpu_r6v.sh r6z_fix 40
