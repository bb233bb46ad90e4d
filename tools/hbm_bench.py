"""HBM-bound kernel microbenchmark at the SDXL 1024^2 b=4 train-step shapes (not a test): each kernel
timed with HIP events (median of reps), reported with its algorithmic bytes and GB/s against the
8 TB/s HBM peak.  One JSON line per (kernel, shape).

usage: python tools/hbm_bench.py [--only gn,ln,geglu,colsum,adamw,attn]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
BF = torch.bfloat16
PEAK = 8000.0


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for i in range(reps):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))
    return ts[len(ts) // 2] * 1e-3


def emit(name, shape, sec, nbytes, flops=None):
    d = {"kernel": name, "shape": shape, "us": round(sec * 1e6, 2), "bytes_MB": round(nbytes / 1e6, 2),
         "GBps": round(nbytes / sec / 1e9, 1), "frac_hbm": round(nbytes / sec / 1e9 / PEAK, 3)}
    if flops:
        d["TFLOPs"] = round(flops / sec / 1e12, 1)
    print(json.dumps(d), flush=True)


def gn(N, H, W, C, silu=True):
    x = torch.randn(N, H, W, C, device=dev).to(BF)
    g, b = torch.ones(C, device=dev, dtype=BF), torch.zeros(C, device=dev, dtype=BF)
    y, st = K.groupnorm_fwd(x, g, b, 32, 1e-5, silu)
    e = x.numel() * 2
    emit("groupnorm_fwd", [N, H, W, C], timeit(lambda: K.groupnorm_fwd(x, g, b, 32, 1e-5, silu, out=y)), 3 * e)
    dy = torch.randn_like(x)
    dx = torch.empty_like(x)
    dg = torch.empty(C, device=dev, dtype=BF)
    db = torch.empty(C, device=dev, dtype=BF)
    emit("groupnorm_bwd", [N, H, W, C], timeit(lambda: K.groupnorm_bwd(x, dy, g, 32, silu, st, dx=dx, dgamma=dg,
                                                                       dbeta=db)), 3 * e)


def ln(R, C):
    x = torch.randn(R, C, device=dev).to(BF)
    g, b = torch.ones(C, device=dev, dtype=BF), torch.zeros(C, device=dev, dtype=BF)
    y, st = K.layernorm_fwd(x, g, b, 1e-5)
    e = x.numel() * 2
    emit("layernorm_fwd", [R, C], timeit(lambda: K.layernorm_fwd(x, g, b, 1e-5, out=y)), 2 * e)
    dy = torch.randn_like(x)
    dx = torch.empty_like(x)
    dg = torch.empty(C, device=dev, dtype=BF)
    db = torch.empty(C, device=dev, dtype=BF)
    emit("layernorm_bwd", [R, C], timeit(lambda: K.layernorm_bwd(x, dy, g, st, dx=dx, dgamma=dg, dbeta=db)), 3 * e)
    dres = torch.randn_like(x)
    emit("layernorm_bwd_res(dx only)", [R, C], timeit(lambda: K.layernorm_bwd_res(x, dy, dres, g, st)), 4 * e)


def geglu(R, F):
    h = torch.randn(R, 2 * F, device=dev).to(BF)
    o = K.geglu_fwd(h)
    emit("geglu_fwd", [R, F], timeit(lambda: K.geglu_fwd(h, out=o)), (2 * F + F) * R * 2)
    d = torch.randn(R, F, device=dev).to(BF)
    emit("geglu_bwd", [R, F], timeit(lambda: K.geglu_bwd(h, d)), (2 * F + F + 2 * F) * R * 2)


def colsum(R, C):
    x = torch.randn(R, C, device=dev).to(BF)
    out = torch.empty(1, C, device=dev, dtype=BF)
    emit("colsum", [R, C], timeit(lambda: K.colsum(x, out=out)), R * C * 2)


def attn(B, N, H, D, Nk=None):
    Nk = Nk or N
    q, k, v = (torch.randn(B, n, H * D, device=dev).to(BF) for n in (N, Nk, Nk))
    o, lse = K.attn_fwd(q, k, v, H)
    fl = 4.0 * B * H * N * Nk * D
    emit("attn_fwd", [B, N, Nk, H, D], timeit(lambda: K.attn_fwd(q, k, v, H, out=o)), 0, fl)
    do = torch.randn_like(o)
    emit("attn_bwd", [B, N, Nk, H, D], timeit(lambda: K.attn_bwd(q, k, v, o, lse, do, H)), 0, 2.5 * fl)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="gn,ln,geglu,colsum,attn")
    a = ap.parse_args()
    only = set(a.only.split(","))
    if "gn" in only:
        for s in [(4, 128, 128, 320), (4, 64, 64, 640), (4, 32, 32, 1280), (4, 128, 128, 960), (4, 32, 32, 2560)]:
            gn(*s)
    if "ln" in only:
        for s in [(16384, 640), (4096, 1280)]:
            ln(*s)
    if "geglu" in only:
        for s in [(16384, 2560), (4096, 5120)]:
            geglu(*s)
    if "colsum" in only:
        for s in [(65536, 320), (16384, 640), (4096, 1280), (16384, 5120), (4096, 10240)]:
            colsum(*s)
    if "attn" in only:
        attn(4, 4096, 10, 64)
        attn(4, 1024, 20, 64)
        attn(4, 4096, 10, 64, 77)
        attn(4, 2381, 24, 128)


if __name__ == "__main__":
    main()
