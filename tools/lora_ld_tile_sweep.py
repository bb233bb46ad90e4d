"""Isolated tile sweep of the fused LoRA GEMMs at the SDXL LoRA (C4) linear shapes (not a test): the forward
(kernels.linear_lora: t = x A^T inside the base GEMM) and the backward input gradient (kernels.linear_dgrad_lora:
u = dy (sB) inside the dgrad) on each fused tile, against the planned dispatch (native host layer: the two-launch
form's tile, 0 -> 4).  HIP-event median of --reps launches; one JSON line per (form, shape).

usage: python tools/lora_ld_tile_sweep.py [--reps 30]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402

BF = torch.bfloat16
TILES = {1: 128, 4: 128, 7: 160, 8: 160}   # fused tiles -> BN
# (M tokens, K in, N out, parts): SDXL level-2 / level-1 sites at 1024^2 b=4 (attn1 q|k|v, to_out, attn2.to_q,
# ff.proj, ff.net.2, proj_in / proj_out)
FWD = [(4096, 1280, 3840, 3), (4096, 1280, 1280, 1), (4096, 1280, 10240, 1), (4096, 5120, 1280, 1),
       (16384, 640, 1920, 3), (16384, 640, 640, 1), (16384, 640, 5120, 1), (16384, 2560, 640, 1)]
DGRAD = [(4096, 1280, 1280, 1), (4096, 10240, 1280, 1), (4096, 1280, 5120, 1), (16384, 640, 640, 1),
         (16384, 5120, 640, 1), (16384, 640, 2560, 1), (4096, 3840, 1280, 3), (16384, 1920, 640, 3)]
# (M, N out = dgrad K, K in = dgrad N, parts along K)


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
    return round(ts[len(ts) // 2] * 1e3, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--ms", default="", help="level-2,level-1 row counts to sweep instead of 4096,16384 (e.g. 4160,16640)")
    a = ap.parse_args()
    if a.ms:
        m2, m1 = (int(v) for v in a.ms.split(","))
        remap = {4096: m2, 16384: m1}
        FWD[:] = [(remap[M], *rest) for M, *rest in FWD]
        DGRAD[:] = [(remap[M], *rest) for M, *rest in DGRAD]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    r = 32

    def rnd(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(BF)

    for M, Kd, N, P in FWD:
        pw = N // P
        x, w = rnd(M, Kd), rnd(N, Kd, scale=0.05)
        down = rnd(P * r, Kd, scale=0.05)
        up2 = torch.zeros(N, P * r, device=dev, dtype=BF)
        for p in range(P):
            up2[p * pw:(p + 1) * pw, p * r:(p + 1) * r] = rnd(pw, r, scale=0.05)
        t = torch.empty(M, P * r, device=dev, dtype=BF)
        res = {"form": "fwd", "M": M, "K": Kd, "N": N, "parts": P,
               "planned_us": timeit(lambda: K.linear_lora(x, w, None, None, down, up2, t, r, pw), a.reps)}
        K.set_lora_fuse(False)
        res["two_launch_us"] = timeit(lambda: K.linear_lora(x, w, None, None, down, up2, t, r, pw), a.reps)
        K.set_lora_fuse(True)
        for tile, bn in TILES.items():
            if pw % bn == 0:
                res[f"tile{tile}_us"] = timeit(lambda: K.linear_lora(x, w, None, None, down, up2, t, r, pw, tile=tile),
                                               a.reps)
        print(json.dumps(res), flush=True)
    for M, Nout, Kin, P in DGRAD:
        pw = Nout // P
        dy, w = rnd(M, Nout), rnd(Nout, Kin, scale=0.05)
        up2 = torch.zeros(Nout, P * r, device=dev, dtype=BF)
        for p in range(P):
            up2[p * pw:(p + 1) * pw, p * r:(p + 1) * r] = rnd(pw, r, scale=0.05)
        down = rnd(P * r, Kin, scale=0.05)
        upT = torch.cat([up2[p * pw:(p + 1) * pw, p * r:(p + 1) * r].t() for p in range(P)], 1).contiguous()
        downT = down.t().contiguous()
        u = torch.empty(M, P * r, device=dev, dtype=BF)
        res = {"form": "dgrad", "M": M, "N_out": Nout, "K_in": Kin, "parts": P,
               "planned_us": timeit(lambda: K.linear_dgrad_lora(dy, w, up2, down, upT, downT, u), a.reps)}
        K.set_lora_fuse(False)
        res["two_launch_us"] = timeit(lambda: K.linear_dgrad_lora(dy, w, up2, down, upT, downT, u), a.reps)
        K.set_lora_fuse(True)
        for tile, bn in TILES.items():
            if Kin % bn == 0:
                res[f"tile{tile}_us"] = timeit(lambda: K.linear_dgrad_lora(dy, w, up2, down, upT, downT, u, tile=tile),
                                               a.reps)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
