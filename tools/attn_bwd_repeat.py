"""Bit-repeatability of the flash attention backward (not a test): for the SDXL ARB level-1/level-2 self-attention
shapes (q, k, v as views of one fused qkv buffer, as the LoRA qkv projection produces them), run K.attn_bwd many times
on identical inputs -- into NaN-prefilled and into stale outputs, with and without a GEMM load on a second stream --
and report, per shape, how many repetitions differ from the first and where (rows / heads of dq, dk, dv).

usage: python tools/attn_bwd_repeat.py [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402

BF = torch.bfloat16


def where(a, b, H, D):
    d = (a.view(torch.int16) != b.view(torch.int16))
    if not d.any():
        return None
    nan = torch.isnan(a.float()).sum().item()
    idx = d.nonzero()
    rows = sorted(set(idx[:, 1].tolist()))
    heads = sorted(set((idx[:, 2] // D).tolist()))
    return f"{d.sum().item()} elems (nan {nan}), batches {sorted(set(idx[:, 0].tolist()))}, rows {rows[:6]}..{rows[-3:]} " \
           f"({len(rows)} rows), heads {heads[:8]}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    side = torch.cuda.Stream(device=dev)
    ga = torch.randn(8192, 5120, device=dev).to(BF)
    gb = torch.randn(5120, 5120, device=dev).to(BF)
    shapes = [(4, 1008, 20, 64), (4, 1040, 20, 64), (4, 1024, 20, 64), (4, 4032, 10, 64), (4, 4160, 10, 64),
              (2, 1008, 20, 64), (1, 300, 4, 64)]
    bad = 0
    for B, N, H, D in shapes:
        torch.manual_seed(1)
        C = H * D
        qkv = (torch.randn(B, N, 3 * C, device=dev) * 2).to(BF)
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        o, lse = K.attn_fwd(q, k, v, H)
        do = torch.randn(B, N, C, device=dev).to(BF)
        d0 = torch.empty_like(qkv)
        r0 = K.attn_bwd(q, k, v, o, lse, do, H, dq=d0[..., :C], dk=d0[..., C:2 * C], dv=d0[..., 2 * C:])
        torch.cuda.synchronize()
        nd = 0
        for rep in range(a.reps):
            mode = rep % 4
            d1 = torch.full_like(qkv, float("nan")) if mode in (0, 2) else d0.clone().mul_(0.999)
            if mode >= 2:
                with torch.cuda.stream(side):
                    for _ in range(3):
                        K.linear(ga, gb)
            r1 = K.attn_bwd(q, k, v, o, lse, do, H, dq=d1[..., :C], dk=d1[..., C:2 * C], dv=d1[..., 2 * C:])
            torch.cuda.synchronize()
            for name, x0, x1 in zip(("dq", "dk", "dv"), r0, r1):
                w = where(x1, x0, H, D)
                if w is not None:
                    nd += 1
                    print(f"  B{B} N{N} H{H} rep {rep} mode {mode} {name}: {w}", flush=True)
        bad += nd
        print(f"B{B} N{N} H{H} D{D}: {nd} differing outputs over {a.reps} reps", flush=True)
    print("TOTAL differing", bad, flush=True)


if __name__ == "__main__":
    main()
