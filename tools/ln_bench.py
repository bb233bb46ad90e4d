"""LayerNorm backward on the SDXL shapes (not a test): round 2's row pass + parameter pass against the
fused single pass (otamd_layernorm_bwd_fused), HIP-event medians per call.

usage: python tools/ln_bench.py [--reps 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402


def timeit(fn, reps):
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
    return ts[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for rows, C in ((4096, 1280), (16384, 640)):
        x = torch.randn(rows, C, device=dev).bfloat16()
        g, b = torch.randn(C, device=dev).bfloat16(), torch.randn(C, device=dev).bfloat16()
        y, st = K.layernorm_fwd(x, g, b, 1e-5)
        dy, dres = torch.randn_like(x), torch.randn_like(x)
        pg, pb = torch.zeros(C, dtype=torch.bfloat16, device=dev), torch.zeros(C, dtype=torch.bfloat16, device=dev)
        t_rows = timeit(lambda: K.layernorm_bwd_res(x, dy, dres, g, st), a.reps)
        t_par = timeit(lambda: K.layernorm_param_grad(x, dy, st, pg, pb), a.reps)
        t_fused = timeit(lambda: K.layernorm_bwd_fused(x, dy, g, st, dres=dres, dgamma=pg, dbeta=pb), a.reps)
        t_fwd = timeit(lambda: K.layernorm_fwd(x, g, b, 1e-5, out=y), a.reps)
        mb = rows * C * 2 / 1e6
        print(json.dumps({"rows": rows, "C": C, "fwd_us": round(t_fwd, 1), "fwd_tbs": round(2 * mb / t_fwd, 2),
                          "rows_us": round(t_rows, 1), "param_us": round(t_par, 1), "fused_us": round(t_fused, 1),
                          "fused_tbs": round(4 * mb / t_fused, 2)}), flush=True)


if __name__ == "__main__":
    main()
