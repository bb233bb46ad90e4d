"""Per-step HBM traffic by kernel family from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of a wide
(16 B/lane) coalesced read, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores.  Both are
memory-side L2 counters, so Infinity-Cache hits are included (an upper bound on HBM bytes).
One step = the dispatches after the second-to-last fused-AdamW (bf16 or f32) launch up to and including the
last one (bench.py's last timed step; the roofline's extra eager GEMM step comes after it and is
excluded by taking the step that ends at the second-to-last AdamW when three or more exist).

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir>
"""
import csv
import glob
import json
import sys


def load(d, counter):
    f = [p for p in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)]
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = {}
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            if r.get("Counter_Name") != counter:
                continue
            did = int(r["Dispatch_Id"])
            rows[did] = (r["Kernel_Name"], rows.get(did, ("", 0.0))[1] + float(r["Counter_Value"]))
    return rows


def family(name):
    if "gemm" in name or "splitk_reduce" in name:
        return "gemm"
    if name.startswith("attn") or "attn_" in name:
        return "attention"
    if "adamw" in name or "grad_sqnorm" in name or "clip_coef" in name:
        return "optimizer"
    if name.startswith(("gn_", "ln_")) or "gn_" in name[:20]:
        return "norm"
    return "other"


def step_window(rows):
    ids = sorted(rows)
    marks = [i for i in ids if "adamw_" in rows[i][0]]   # bf16 (full fine-tune) or f32 (LoRA) update
    if len(marks) >= 3:
        lo, hi = marks[-3], marks[-2]
    else:
        lo, hi = marks[-2], marks[-1]
    return [i for i in ids if lo < i <= hi]


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for label, rows, scale in (("read", fetch, 2.0), ("write", write, 1.0)):
        win = step_window(rows)
        fam, launches = {}, {}
        for i in win:
            name, v = rows[i]
            k = family(name)
            fam[k] = fam.get(k, 0.0) + v * 1024.0 * scale   # FETCH_SIZE / WRITE_SIZE are in KiB
            launches[k] = launches.get(k, 0) + 1
        out[label] = {k: round(v / 1e9, 3) for k, v in fam.items()}
        out[label + "_launches"] = launches
    out["unit"] = "GB per train step of the profiled bench config, FETCH_SIZE x 2 + WRITE_SIZE"
    g = out["read"].get("gemm", 0.0) + out["write"].get("gemm", 0.0)
    out["gemm_total_gb"] = round(g, 3)
    out["gemm_launches"] = out["read_launches"].get("gemm", 0)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
