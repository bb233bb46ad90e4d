# Round 6: isolated sweep of the 4-wave 128x160 (11) / 128x128 (12) tiles against the 8-wave ones on the level-1/2 shapes.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
S=fwd:4096:1280:1280,dgrad:4096:1280:1280,fwd:4096:10240:1280,fwd:4096:1280:5120,dgrad:4096:5120:1280,dgrad:4096:1280:3840,fwd:4096:3840:1280,fwd:16384:640:640,dgrad:16384:640:640,wgrad:1280:1280:4096
timeout -k 10 400 python -u tools/gemm_tile_sweep.py --shapes $S --plans 7:1,11:1,4:1,12:1,0:1,8:1 > gpurun_out/r6_tiles_w4.jsonl 2> gpurun_out/r6_tiles_w4.err || { tail -20 gpurun_out/r6_tiles_w4.err; exit 1; }
cat gpurun_out/r6_tiles_w4.jsonl
