"""LayerNorm kernels at the SDXL step's shapes, alone: forward, backward (+ residual gradient), parameter gradients.
HIP-event time per call, cold (the Infinity Cache flushed by a 512 MiB write before each call, as in the step where
other kernels ran in between) and warm; algorithmic bytes / time.  Not a test.

    python tools/ln_bench.py [--reps 20] [--out gpurun_out/ln_bench.jsonl]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402

SHAPES = [(4096, 1280), (16384, 640)]   # SDXL 1024^2 b=4: level-3 and level-2 transformer rows


def timed(fn, reps, flush):
    ts = []
    for _ in range(reps):
        if flush is not None:
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/ln_bench.jsonl")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    flush = torch.zeros(128 << 20, device=dev)   # 512 MiB
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        for rows, C in SHAPES:
            g = torch.Generator(device=dev).manual_seed(rows + C)
            x = torch.randn(rows, C, device=dev, generator=g).bfloat16()
            dy = torch.randn(rows, C, device=dev, generator=g).bfloat16()
            dres = torch.randn(rows, C, device=dev, generator=g).bfloat16()
            gamma = (1 + 0.1 * torch.randn(C, device=dev, generator=g)).bfloat16()
            beta = (0.1 * torch.randn(C, device=dev, generator=g)).bfloat16()
            y, stats = K.layernorm_fwd(x, gamma, beta, 1e-5)
            dg = torch.empty(C, device=dev)
            db = torch.empty(C, device=dev)
            E = rows * C * 2
            cases = {
                "fwd": (lambda: K.layernorm_fwd(x, gamma, beta, 1e-5), 2 * E),
                "bwd_res": (lambda: K.layernorm_bwd_res(x, dy, dres, gamma, stats), 4 * E),
                "param_grad": (lambda: K.layernorm_param_grad(x, dy, stats, dg, db), 2 * E),
                "bwd_res+param": (lambda: (K.layernorm_bwd_res(x, dy, dres, gamma, stats),
                                           K.layernorm_param_grad(x, dy, stats, dg, db)), 4 * E),
            }
            for name, (fn, nbytes) in cases.items():
                fn()
                torch.cuda.synchronize()
                cold = timed(fn, a.reps, flush)
                warm = timed(fn, a.reps, None)
                r = {"op": name, "rows": rows, "C": C, "us_cold": round(cold, 2), "us_warm": round(warm, 2),
                     "GBps_cold": round(nbytes / cold / 1e3, 1), "GBps_warm": round(nbytes / warm / 1e3, 1)}
                print(json.dumps(r), flush=True)
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
