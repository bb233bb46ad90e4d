"""Flash-attention kernel timings on the SDXL / Flux attention shapes (not a test).

Prints one JSON line per shape: fwd and bwd (dQ + dK/dV (+ cast)) wall time per call from HIP
events over `--reps` back-to-back calls, and TF/s against the algorithmic work (fwd 4 Nq Nk D per
(image, head); bwd 2 x fwd).  OTAMD_LIB_ALT selects the
builds to compare.

usage: python tools/attn_bench.py [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402

SHAPES = [  # (B, Nq, Nk, H, D, calls per SDXL 1024^2 b=4 step)
    (4, 4096, 4096, 10, 64, 10), (4, 1024, 1024, 20, 64, 60), (4, 4096, 77, 10, 64, 10), (4, 1024, 77, 20, 64, 60),
    (4, 2381, 2381, 24, 128, 57),
]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    tot_f = tot_b = 0.0
    for B, Nq, Nk, H, D, calls in SHAPES:
        q = torch.randn(B, Nq, H * D, device=dev).to(torch.bfloat16)
        k = torch.randn(B, Nk, H * D, device=dev).to(torch.bfloat16)
        v = torch.randn(B, Nk, H * D, device=dev).to(torch.bfloat16)
        do = torch.randn(B, Nq, H * D, device=dev).to(torch.bfloat16)
        o, lse = K.attn_fwd(q, k, v, H)
        dq, dk, dv = K.attn_bwd(q, k, v, o, lse, do, H)
        tf = timeit(lambda: K.attn_fwd(q, k, v, H, out=o), args.reps)
        tb = timeit(lambda: K.attn_bwd(q, k, v, o, lse, do, H, dq=dq, dk=dk, dv=dv), args.reps)
        fl = 4.0 * B * H * Nq * Nk * D
        if calls and D == 64:
            tot_f += tf * calls
            tot_b += tb * calls
        print(json.dumps({"shape": [B, Nq, Nk, H, D], "fwd_us": round(tf, 1), "fwd_tflops": round(fl / tf / 1e6, 1),
                          "bwd_us": round(tb, 1), "bwd_tflops": round(2 * fl / tb / 1e6, 1)}), flush=True)
    print(json.dumps({"sdxl_step_ms": {"fwd": round(tot_f / 1e3, 2), "bwd": round(tot_b / 1e3, 2)}}), flush=True)


if __name__ == "__main__":
    main()
