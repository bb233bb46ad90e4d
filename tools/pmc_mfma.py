"""MFMA utilisation per kernel family from one rocprofv3 --pmc pass
(SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES).

Units (MI355X_MICROARCH.md, per-instruction constants / DVFS rows):
  * SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles summed over every SIMD of the chip
    (= 32 x N_mfma for v_mfma_f32_32x32x16_bf16, 16 x N for 16x16x32), i.e. 1024 bf16 FLOP per
    busy cycle -> counter FLOP = busy x 1024;
  * GRBM_GUI_ACTIVE is summed over the 8 XCDs: per-XCD busy cycles = GRBM / 8, so the chip had
    GRBM / 8 x 1024 SIMD-cycles available and util = busy / (GRBM x 128).
One step is the window that ends at the second-to-last fused-AdamW dispatch (pmc_traffic.step_window).

usage: python tools/pmc_mfma.py <pmc_dir> [<out.json>]
"""
import csv
import glob
import json
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import family, step_window  # noqa: E402


def load(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = defaultdict(lambda: {"name": "", "c": defaultdict(float)})
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            did = int(r["Dispatch_Id"])
            rows[did]["name"] = r["Kernel_Name"]
            rows[did]["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    return rows


def main():
    rows = load(sys.argv[1])
    win = step_window({k: (v["name"], 0.0) for k, v in rows.items()})
    fam = defaultdict(lambda: defaultdict(float))
    kern = defaultdict(lambda: defaultdict(float))
    for i in win:
        r = rows[i]
        f = family(r["name"])
        short = r["name"].split("(")[0][:90]
        for dst in (fam[f], kern[short]):
            dst["busy"] += r["c"].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
            dst["grbm"] += r["c"].get("GRBM_GUI_ACTIVE", 0.0)
            dst["cu_busy"] += r["c"].get("SQ_BUSY_CU_CYCLES", 0.0)
            dst["launches"] += 1

    def summarise(d):
        out = {}
        for k, v in sorted(d.items(), key=lambda kv: -kv[1]["grbm"]):
            out[k] = {"launches": int(v["launches"]),
                      "mfma_tflop_counted": round(v["busy"] * 1024 / 1e12, 3),
                      "mfma_util": round(v["busy"] / (v["grbm"] * 128), 4) if v["grbm"] else None,
                      "grbm_gui_active": v["grbm"], "sq_busy_cu_cycles": v["cu_busy"]}
        return out

    res = {"unit": "per train step; mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 XCD x 1024 SIMDs)",
           "families": summarise(fam), "kernels": dict(list(summarise(kern).items())[:40])}
    tot_b = sum(v["busy"] for v in fam.values())
    tot_g = sum(v["grbm"] for v in fam.values())
    res["all_kernels_mfma_util"] = round(tot_b / (tot_g * 128), 4) if tot_g else None
    s = json.dumps(res, indent=1)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            fh.write(s)
    print(s)


if __name__ == "__main__":
    main()
