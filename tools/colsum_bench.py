"""Per-group column sums (the conv bias / time-embedding drow reductions) at the SDXL step's shapes, alone.
HIP-event median time per call with the Infinity Cache flushed before each call; algorithmic bytes / time.  Not a test.

    python tools/colsum_bench.py [--reps 30]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402

SHAPES = [(4, 16384, 320), (4, 4096, 640), (4, 1024, 1280), (1, 65536, 320), (1, 1024, 2560)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    flush = torch.zeros(128 << 20, device=dev)
    for groups, rows, C in SHAPES:
        x = torch.randn(groups * rows, C, device=dev).bfloat16()
        K.colsum(x, rows)
        ts = []
        for _ in range(a.reps):
            flush.add_(1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            K.colsum(x, rows)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        us = ts[len(ts) // 2]
        print(json.dumps({"groups": groups, "rows": rows, "C": C, "us": round(us, 2),
                          "GBps": round(x.numel() * 2 / us / 1e3, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
