# bench.py --gpus 2 (two gloo ranks on the one GPU) run directly, twice, with the ranks' output in files
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp OTAMD_DIST_BACKEND=gloo
for i in 1 2; do
  date +%T
  timeout -k 10 170 python -u bench.py --gpus 2 --steps 2 --warmup 1 --res 256 --batch 1 --no-cpu-baseline --no-vae > gpurun_out/r4two_$i.out 2> gpurun_out/r4two_$i.err; rc=$?
  date +%T
  echo "run $i rc=$rc"; tail -3 gpurun_out/r4two_$i.err; cat gpurun_out/r4two_$i.out | cut -c1-200
  [ $rc -eq 0 ] || exit 1
done
