set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py::test_attention tests/test_bench_gpu.py "tests/test_dp_gpu.py::test_rccl_reducer_world1" \
  tests/test_host_layer_gpu.py tests/test_fullsize_gpu.py::test_full_unet_matches_oracle > gpurun_out/r4a_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r4a_tests.log
exit $rc
