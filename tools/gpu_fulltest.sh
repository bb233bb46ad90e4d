# The whole -m gpu suite in one process (as the driver runs it), log under gpurun_out/.  usage: bash tools/gpu_fulltest.sh <tag>
set -o pipefail
TAG=${1:-full}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/gputest_$TAG.log | tail -3
[ $rc -ne 0 ] && grep -E "FAILED|Error" gpurun_out/gputest_$TAG.log | head -20
exit $rc
