"""Per-launch-shape kernel durations from a rocprofv3 --kernel-trace CSV or results .db (not a test): groups launches by
(kernel name, grid, LDS bytes) and prints count / average / minimum duration in microseconds, so kernels
launched at several problem sizes (attention at 4096 / 1024 / 77 keys) are told apart.

usage: python tools/ktrace_by_grid.py <kernel_trace.csv | results.db | dir> [--match attn] [--top 40]
"""
import argparse
import collections
import csv
import glob
import os
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path", help="kernel_trace.csv, or a directory searched for one")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    path = args.path
    if os.path.isdir(path):
        found = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) +
                       glob.glob(os.path.join(path, "**", "*.db"), recursive=True))
        path = found[-1]
    agg = collections.defaultdict(list)

    def add(name, grid, wg, lds, dur):
        if args.match in name:
            agg[(name.split("(")[0], tuple(g // max(1, w) for g, w in zip(grid, wg)), lds)].append(dur)

    if path.endswith(".db"):
        con = sqlite3.connect(path)
        for r in con.execute("select name, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, workgroup_z, lds_size, "
                             "start, end from kernels"):
            add(r[0], r[1:4], r[4:7], int(r[7] or 0), (r[9] - r[8]) / 1e3)
    else:
        with open(path) as f:
            for row in csv.DictReader(f):
                add(row["Kernel_Name"], [int(row[f"Grid_Size_{c}"]) for c in "XYZ"],
                    [int(row[f"Workgroup_Size_{c}"]) for c in "XYZ"],
                    int(row.get("LDS_Block_Size", row.get("Lds_Size", 0)) or 0),
                    (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:args.top]
    for (name, grid, lds), d in rows:
        d.sort()
        print(f"{name[:48]:48s} grid={grid!s:18s} lds={lds:6d} n={len(d):5d} avg={sum(d) / len(d):9.2f} "
              f"p50={d[len(d) // 2]:9.2f} min={d[0]:9.2f} us")


if __name__ == "__main__":
    main()
