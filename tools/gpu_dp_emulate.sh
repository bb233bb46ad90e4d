# RCCL footprint emulation on one GPU (trainer/ddp.py OTAMD_DP_EMULATE): the SDXL step with each 256 MB gradient
# bucket's ring all-reduce replaced by a paced copy kernel on the reducer's issue stream, against the plain step,
# interleaved on one box.  usage: bash tools/gpu_dp_emulate.sh
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-vae --steps 15 --warmup 4 > gpurun_out/dpemu_$tag.json 2> gpurun_out/dpemu_$tag.err || { tail -5 gpurun_out/dpemu_$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/dpemu_$tag.json')); print('$tag', d['ms_per_step'], d['step_ms_p50'], d['loss'])"
}
for rep in 1 2; do
  run base_$rep OTAMD_DP_EMULATE=0 &&
  run n8_c64_g400_$rep OTAMD_DP_EMULATE=8 OTAMD_DP_EMULATE_CUS=64 OTAMD_DP_EMULATE_GBS=400 &&
  run n8_c32_g300_$rep OTAMD_DP_EMULATE=8 OTAMD_DP_EMULATE_CUS=32 OTAMD_DP_EMULATE_GBS=300 &&
  run n8_c64_g600_$rep OTAMD_DP_EMULATE=8 OTAMD_DP_EMULATE_CUS=64 OTAMD_DP_EMULATE_GBS=600 || exit 1
done
