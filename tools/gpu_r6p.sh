# Round 6: C4 run-to-run determinism, the current library against the previous commit's (native host path in both: the
# old library in a copy of the tree), per-step losses in full precision.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
ROOT=$(pwd)
rm -rf /tmp/altrepo && mkdir /tmp/altrepo && cp -r bench.py onetrainer_amd oracle tools /tmp/altrepo/ && cp onetrainer_amd/_lib/libotamd_head.so /tmp/altrepo/onetrainer_amd/_lib/libotamd.so
run() {  # name, dir
  local name=$1 dir=$2
  (cd $dir && timeout -k 10 200 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae --steps 5 --warmup 2 > $ROOT/gpurun_out/r6p.json 2> $ROOT/gpurun_out/r6p.err) || { echo "$name failed"; tail -5 gpurun_out/r6p.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6p.json')); print('$name', ' '.join(repr(v) for v in d['losses_exact']))"
}
for rep in 1 2 3 4 5 6 7 8; do
  run cur $ROOT
  run prev /tmp/altrepo
done
