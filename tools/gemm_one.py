"""One GEMM shape launched repeatedly (for rocprofv3 PMC passes and per-launch timing; not a test).

usage: python tools/gemm_one.py <fwd|dgrad|wgrad> M N K [--tile T --splits S] [--reps 50]
  fwd   y[M,N]  = x[M,K] w[N,K]^T          (A K-mode, B K-mode)
  dgrad dx[M,N] = dy[M,K] w[K,N]           (A K-mode, B MN-mode)
  wgrad dw[M,N] = dy[K,M]^T x[K,N]         (A MN-mode, B MN-mode; K = tokens)
Prints the median launch time and TFLOP/s (HIP events), and torch.matmul's for the same product.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("op")
ap.add_argument("M", type=int)
ap.add_argument("N", type=int)
ap.add_argument("K", type=int)
ap.add_argument("--tile", type=int, default=None)
ap.add_argument("--splits", type=int, default=1)
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--torch", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
BF = torch.bfloat16
M, N, Kd = a.M, a.N, a.K
g = torch.Generator(device=dev).manual_seed(0)
if a.op == "fwd":
    x = torch.randn(M, Kd, device=dev, generator=g).to(BF)
    w = (torch.randn(N, Kd, device=dev, generator=g) * 0.05).to(BF)
    fn, ref, key = (lambda: K.linear(x, w)), (lambda: x @ w.t()), (0, 0, M, N, Kd)
elif a.op == "dgrad":
    x = torch.randn(M, Kd, device=dev, generator=g).to(BF)
    w = (torch.randn(Kd, N, device=dev, generator=g) * 0.05).to(BF)
    fn, ref, key = (lambda: K.linear_dgrad(x, w)), (lambda: x @ w), (0, 1, M, N, Kd)
else:
    dy = torch.randn(Kd, M, device=dev, generator=g).to(BF)
    x = torch.randn(Kd, N, device=dev, generator=g).to(BF)
    out = torch.empty(M, N, device=dev, dtype=BF)
    fn, ref, key = (lambda: K.linear_wgrad(dy, x, out=out)), (lambda: dy.t() @ x), (1, 1, M, N, Kd)
if a.tile is not None:
    os.environ["OTAMD_GEMM_PLAN"] = ",".join(map(str, key)) + f":{a.tile}:{a.splits}"
    K._PLAN_OVERRIDES = None


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


fl = 2.0 * M * N * Kd
t = timeit(fn, a.reps)
r = {"op": a.op, "M": M, "N": N, "K": Kd, "tile": a.tile, "splits": a.splits, "us": round(t * 1e6, 1),
     "tflops": round(fl / t / 1e12, 1)}
if a.torch:
    tt = timeit(ref, a.reps)
    r["torch_us"], r["torch_tflops"] = round(tt * 1e6, 1), round(fl / tt / 1e12, 1)
print(json.dumps(r), flush=True)
