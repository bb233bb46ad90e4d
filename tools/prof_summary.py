"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) into a per-kernel stats CSV.

usage: python tools/prof_summary.py gpurun_out/prof/run_results.db profiles/<name>.csv [--steps-kernel adamw]

Columns: Name, Calls, TotalDurationNs, AverageNs, Percentage, CallsPerStep, MsPerStep.  "Per step"
divides by the number of launches of the kernel whose name contains --steps-kernel (the fused
optimizer runs exactly once per train step), so warmup steps are included in the normalisation.
"""
from __future__ import annotations

import argparse
import csv
import sqlite3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("out")
    ap.add_argument("--steps-kernel", default="adamw_bf16")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--all", action="store_true", help="every dispatch of the run (default: the timed steps only)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    if a.all:
        rows = c.execute("select name, count(*), sum(duration) from kernels group by name order by sum(duration) desc").fetchall()
        steps = sum(r[1] for r in rows if a.steps_kernel in r[0]) or 1
    else:
        # only whole steps between optimizer launches, skipping the first window (model init, first-shape
        # planning, warm-up) and the last two (bench.py's two extra roofline steps run after the timed steps)
        ev = c.execute("select name, start, end from kernels order by start").fetchall()
        marks = [s for n, s, e in ev if a.steps_kernel in n]
        lo, hi = marks[1], marks[-3]
        steps = max(1, len(marks) - 4)
        agg = {}
        for n, s, e in ev:
            if lo < s <= hi:
                cnt, d = agg.get(n, (0, 0))
                agg[n] = (cnt + 1, d + (e - s))
        rows = sorted(((n, cnt, d) for n, (cnt, d) in agg.items()), key=lambda r: -r[2])
    total = sum(r[2] for r in rows)
    with open(a.out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "CallsPerStep", "MsPerStep"])
        for name, n, dur in rows:
            w.writerow([name, n, dur, round(dur / n, 1), round(100.0 * dur / total, 3), round(n / steps, 2),
                        round(dur / steps / 1e6, 3)])
    print(f"{len(rows)} kernels, {steps} steps, {total / steps / 1e6:.2f} ms GPU time per step")
    for name, n, dur in rows[:a.top]:
        print(f"{dur / steps / 1e6:8.3f} ms/step {n / steps:7.1f}x {dur / n / 1e3:9.1f} us  {name[:110]}")


if __name__ == "__main__":
    main()
