"""HBM-bound elementwise kernels of the SDXL step, alone: GEGLU forward / backward at the level-3 and level-2 FF
shapes (SDXL 1024^2 b=4).  HIP-event median per call with the Infinity Cache flushed first; algorithmic bytes /
time.  Not a test.

    python tools/ew_bench.py [--reps 30]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402


def timed(fn, reps, flush):
    ts = []
    for _ in range(reps):
        flush.add_(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    flush = torch.zeros(128 << 20, device=dev)
    for M, F_ in ((4096, 5120), (16384, 2560)):
        h = torch.randn(M, 2 * F_, device=dev).bfloat16()
        d = torch.randn(M, F_, device=dev).bfloat16()
        E = M * F_ * 2
        for name, fn, nbytes in (("geglu_fwd", lambda: K.geglu_fwd(h), 3 * E),
                                 ("geglu_bwd", lambda: K.geglu_bwd(h, d), 5 * E)):
            fn()
            torch.cuda.synchronize()
            us = timed(fn, a.reps, flush)
            print(json.dumps({"op": name, "M": M, "F": F_, "us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1)}),
                  flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
