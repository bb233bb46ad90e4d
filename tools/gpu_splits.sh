set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out && rm -rf gpurun_out/splits
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/splits -o run -- python -u tools/gemm_splits.py > gpurun_out/splits.log 2>&1 || { echo "probe failed"; tail -30 gpurun_out/splits.log; exit 1; }
DB=$(find gpurun_out/splits -name '*.db' | head -1)
python tools/gemm_splits.py --db "$DB"
