# Build K-loop timing ablations of the GEMM engine (gemm2_kernel.h OTAMD_GEMM_ABL) as onetrainer_amd/_lib/libotamd_abl<N>.so
# from the working tree (select with OTAMD_LIB_ALT=abl<N>; results are garbage, timings are the point).
# usage: bash tools/gemm_ablate.sh 1 2 3 4
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
for N in "$@"; do
  W=$(mktemp -d)
  pids=()
  for f in "$ROOT"/onetrainer_amd/csrc/*.hip; do
    b=$(basename "$f" .hip)
    extra=""
    case "$b" in adamw|diffusion) extra="-ffp-contract=off";; attention) extra="-fno-honor-nans -fno-slp-vectorize";; esac
    "$HIPCC" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -DOTAMD_GEMM_ABL=$N -I "$ROOT/onetrainer_amd/csrc" -c "$f" -o "$W/$b.o" $extra &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait "$p"; done
  "$HIPCC" --offload-arch=gfx950 -shared -fPIC -o "$ROOT/onetrainer_amd/_lib/libotamd_abl$N.so" "$W"/*.o
  rm -rf "$W"
  echo "built libotamd_abl$N.so"
done
