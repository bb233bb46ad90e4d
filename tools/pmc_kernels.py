"""Per-kernel averages of every counter in a rocprofv3 --pmc csv run (not a test).
usage: python tools/pmc_kernels.py <pmc_dir>"""
import csv
import glob
import sys
from collections import defaultdict

f = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
if not f:
    raise SystemExit("no counter_collection.csv")
per = defaultdict(lambda: defaultdict(float))
names = {}
with open(f[0]) as fh:
    for r in csv.DictReader(fh):
        did = int(r["Dispatch_Id"])
        names[did] = r["Kernel_Name"].split("(")[0][:60]
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(int)
for did, c in per.items():
    n = names[did]
    cnt[n] += 1
    for k, v in c.items():
        agg[n][k] += v
for n in sorted(agg, key=lambda n: -agg[n].get("SQ_WAVE_CYCLES", 0)):
    print(n, cnt[n], " ".join(f"{k}={v / cnt[n]:.4g}" for k, v in sorted(agg[n].items())))
