"""Run-to-run determinism of the attention kernels (not a test): the same inputs through attn_fwd / attn_bwd
`--reps` times, every output compared bit for bit with the first call's.  Prints one line per shape and output.

usage: python tools/attn_determinism.py [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402

SHAPES = [(4, 1024, 77, 20, 64), (4, 4096, 77, 10, 64), (1, 100, 77, 3, 64), (2, 1024, 96, 20, 64),
          (4, 1024, 1024, 20, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    bad = 0
    for B, Nq, Nk, H, D in SHAPES:
        q = torch.randn(B, Nq, H * D, device=dev).bfloat16()
        k = torch.randn(B, Nk, H * D, device=dev).bfloat16()
        v = torch.randn(B, Nk, H * D, device=dev).bfloat16()
        do = torch.randn(B, Nq, H * D, device=dev).bfloat16()
        ref = None
        diffs = [0] * 5
        for _ in range(args.reps):
            o, lse = K.attn_fwd(q, k, v, H)
            dq, dk, dv = K.attn_bwd(q, k, v, o, lse, do, H)
            outs = [t.clone() for t in (o, lse, dq, dk, dv)]
            if ref is None:
                ref = outs
            else:
                for i, (a, b) in enumerate(zip(ref, outs)):
                    diffs[i] += int(not torch.equal(a, b))
        torch.cuda.synchronize()
        print((B, Nq, Nk, H, D), dict(zip(("o", "lse", "dq", "dk", "dv"), diffs)), flush=True)
        bad += sum(diffs)
    print("nondeterministic outputs:", bad)


if __name__ == "__main__":
    main()
