# Round 6: stream-hazard probe of the SDXL LoRA step at 1024^2 (b=2, 2 steps), and 6 C3 runs with exact losses.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/hazard_probe.py --model sdxl-lora --res 1024 --batch 2 --steps 2 > gpurun_out/hz_lora1024.txt 2>&1; rc=$?
echo "hazard probe rc=$rc"; grep -v amdgpu.ids gpurun_out/hz_lora1024.txt | head -30
[ $rc -le 1 ] || exit 1
for rep in 1 2 3 4 5 6; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-vae --steps 4 --warmup 2 > gpurun_out/r6r.json 2> gpurun_out/r6r.err || { tail -5 gpurun_out/r6r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6r.json')); print('sdxl $rep', ' '.join(repr(v) for v in d['losses_exact']))"
done
