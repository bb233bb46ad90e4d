# round 5: stream hazard probe (aten + kernel entry points) on the tiny, SD 1.5 and SDXL steps
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for m in "sdxl --res 512" "sd15 --res 512" "sdxl-lora --res 512"; do
  tag=$(echo $m | cut -d' ' -f1)
  timeout -k 10 240 python -u tools/hazard_probe.py --model $m --batch 1 --steps 1 > gpurun_out/hz_$tag.txt 2>&1; rc=$?
  echo "== $m rc=$rc"; grep -v amdgpu.ids gpurun_out/hz_$tag.txt | head -30
  [ $rc -le 1 ] || exit 1
done
