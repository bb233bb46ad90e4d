"""Launch the GEMM ablation shapes back to back (for rocprofv3 --kernel-trace; not a test): each shape with a pinned
(tile, split-K) through OTAMD_GEMM_PLAN, `--reps` launches.  Pair with tools/gemm_ablate.sh (OTAMD_LIB_ALT=abl<N>).

usage: python tools/gemm_abl_run.py [--reps 30]
"""
import argparse
import os
import sys

SHAPES = [  # (op, M, N, K, tile, splits): the SDXL step's level-2 workhorses and a square reference
    ("fwd", 4096, 1280, 1280, 7, 1), ("fwd", 4096, 1280, 1280, 4, 1), ("dgrad", 4096, 1280, 1280, 4, 1),
    ("fwd", 4096, 10240, 1280, 4, 1), ("dgrad", 4096, 1280, 10240, 0, 3), ("fwd", 16384, 5120, 640, 0, 1),
    ("fwd", 4096, 4096, 4096, 0, 1),
]
KEY = {"fwd": (0, 0), "dgrad": (0, 1)}
os.environ["OTAMD_GEMM_PLAN"] = ";".join(f"{KEY[o][0]},{KEY[o][1]},{M},{N},{Kd}:{t}:{s}" for o, M, N, Kd, t, s in SHAPES)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for op, M, N, Kd, t, s in SHAPES:
        x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, Kd, device=dev, generator=g) * 0.05).bfloat16() if op == "fwd" else \
            (torch.randn(Kd, N, device=dev, generator=g) * 0.05).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        f = (lambda: K.linear(x, w, out=out)) if op == "fwd" else (lambda: K.linear_dgrad(x, w, out=out))
        for _ in range(a.reps):
            f()
        torch.cuda.synchronize()
        print(op, M, N, Kd, "tile", t, "splits", s, flush=True)


if __name__ == "__main__":
    main()
