"""Isolated (tile, split-K) sweep of GEMM shapes in one process (not a test): every candidate is checked against the
first candidate's output (bf16 rounding of the fp32 sums; split-K only changes their order) and timed as the median
of --reps launches with HIP events.

usage: python tools/gemm_tile_sweep.py --shapes fwd:4096:1280:1280,dgrad:4096:1280:1280 --plans 7:1,11:1,4:1,12:1
  fwd   y[M,N]  = x[M,K] w[N,K]^T   dgrad dx[M,N] = dy[M,K] w[K,N]   wgrad dw[M,N] = dy[K,M]^T x[K,N]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", required=True)
ap.add_argument("--plans", required=True, help="tile:splits,...")
ap.add_argument("--reps", type=int, default=40)
a = ap.parse_args()
dev = torch.device("cuda:0")
BF = torch.bfloat16


def timeit(f, reps):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for i in range(reps):
        f()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))
    return ts[len(ts) // 2] * 1e-3


for spec in a.shapes.split(","):
    op, M, N, Kd = spec.split(":")
    M, N, Kd = int(M), int(N), int(Kd)
    g = torch.Generator(device=dev).manual_seed(0)
    if op == "fwd":
        x = torch.randn(M, Kd, device=dev, generator=g).to(BF)
        w = (torch.randn(N, Kd, device=dev, generator=g) * 0.05).to(BF)
        fn, key = (lambda: K.linear(x, w)), (0, 0, M, N, Kd)
    elif op == "dgrad":
        x = torch.randn(M, Kd, device=dev, generator=g).to(BF)
        w = (torch.randn(Kd, N, device=dev, generator=g) * 0.05).to(BF)
        fn, key = (lambda: K.linear_dgrad(x, w)), (0, 1, M, N, Kd)
    else:
        dy = torch.randn(Kd, M, device=dev, generator=g).to(BF)
        x = torch.randn(Kd, N, device=dev, generator=g).to(BF)
        fn, key = (lambda: K.linear_wgrad(dy, x, out=torch.empty(M, N, device=dev, dtype=BF))), (1, 1, M, N, Kd)
    ref = None
    for plan in a.plans.split(","):
        t, s = (int(v) for v in plan.split(":"))
        K._PLAN_OVERRIDES = {key: (t, s)}
        y = fn().float()
        if ref is None:
            ref = y
        err = ((y - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()
        us = timeit(fn, a.reps) * 1e6
        print(json.dumps({"op": op, "M": M, "N": N, "K": Kd, "tile": t, "splits": s, "us": round(us, 1),
                          "tflops": round(2.0 * M * N * Kd / us / 1e6, 1), "rel_maxdiff_vs_first": round(err, 5)}),
              flush=True)
    K._PLAN_OVERRIDES = None
