# Build the HIP library from the csrc/ of another git revision as onetrainer_amd/_lib/libotamd_<name>.so
# (selected at run time with OTAMD_LIB_ALT=<name>; A/B of kernel changes inside one GPU call).
# usage: bash tools/ab_lib.sh <git-rev | WT> <name>
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d)
if [ "$REV" = "WT" ]; then   # the working tree's sources (uncommitted edits), e.g. to A/B them against the built library
  mkdir -p "$W/onetrainer_amd" && cp -r "$ROOT/onetrainer_amd/csrc" "$W/onetrainer_amd/"
else
  git -C "$ROOT" archive "$REV" onetrainer_amd/csrc | tar -x -C "$W"
fi
mkdir -p "$W/obj"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
pids=()
for f in "$W"/onetrainer_amd/csrc/*.hip; do
  b=$(basename "$f" .hip)
  extra=""
  case "$b" in adamw|diffusion) extra="-ffp-contract=off";; attention) extra="-fno-honor-nans -fno-slp-vectorize";; esac
  "$HIPCC" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -I "$W/onetrainer_amd/csrc" -c "$f" -o "$W/obj/$b.o" $extra &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
"$HIPCC" --offload-arch=gfx950 -shared -fPIC -o "$ROOT/onetrainer_amd/_lib/libotamd_$NAME.so" "$W"/obj/*.o
rm -rf "$W"
echo "built onetrainer_amd/_lib/libotamd_$NAME.so from $REV"
