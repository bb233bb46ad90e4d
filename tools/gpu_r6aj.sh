# Round 6: per-step times by aspect bucket, C4 with the fused-LoRA tile table (1) and without its exact-M rows (3)
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for v in 1 3; do
  OTAMD_LORA_PLANS=$v timeout -k 10 400 python -u bench.py --model sdxl-lora --no-cpu-baseline --no-vae --steps 28 > gpurun_out/r6aj_$v.json 2> gpurun_out/r6aj.err || { tail -20 gpurun_out/r6aj.err; exit 1; }
done
python3 - <<'PY'
import json, collections
for v in (1, 3):
    d = json.load(open(f"gpurun_out/r6aj_{v}.json"))
    by = collections.defaultdict(list)
    for b, t in zip(d["step_buckets"], d["step_ms_each"]):
        by[tuple(b)].append(t)
    print("plans", v, d["ms_per_step"], {f"{k[0]}x{k[1]}": [min(x), max(x), len(x)] for k, x in sorted(by.items())})
PY
