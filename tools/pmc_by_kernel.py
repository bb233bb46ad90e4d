"""Average PMC counter values per (kernel, grid) from a rocprofv3 --pmc counter_collection.csv (not a test).

usage: python tools/pmc_by_kernel.py <dir or csv> [--match attn]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--match", default="")
    args = ap.parse_args()
    path = args.path
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True))[-1]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if args.match not in name:
                continue
            grid = row.get("Grid_Size", "")
            vals[(name.split("(")[0], grid)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for (name, grid), cs in sorted(vals.items()):
        parts = " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items()))
        print(f"{name[:44]:44s} grid={grid:>10s} {parts}")


if __name__ == "__main__":
    main()
