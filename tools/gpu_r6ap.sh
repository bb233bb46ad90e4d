# Round 6: final check after the exact-row LoRA entries -- LoRA GPU tests, smoke, C4 bench line
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_lora_fused_gpu.py tests/test_lora_gpu.py tests/test_defer_reduce_gpu.py "tests/test_fullsize_gpu.py::test_full_width_sdxl_lora_r32_matches_oracle" > gpurun_out/r6ap_tests.txt 2>&1 || { tail -30 gpurun_out/r6ap_tests.txt; exit 1; }
tail -1 gpurun_out/r6ap_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6ap_smoke.log 2>&1 || { tail -20 gpurun_out/r6ap_smoke.log; exit 1; }
tail -1 gpurun_out/r6ap_smoke.log | cut -c1-120
timeout -k 10 400 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae > gpurun_out/r6ap_bench_sdxl-lora.json 2> gpurun_out/r6ap.err || { tail -20 gpurun_out/r6ap.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6ap_bench_sdxl-lora.json')); print('sdxl-lora', d['value'], d['ms_per_step'], d['step_ms_p50'])"
