"""Skinny-N GEMM (gemm_skinny_kernel, otamd_gemm_set_skinny) against the split-K tile plans on the LoRA
down-projection shapes of the C4 / C5 steps: t = x A^T (K = in features) and u = dy (s B) (K = out features, B as a
K-mode transposed shadow).  Same process, interleaved rounds, HIP events; outputs compared with fp32 torch.  Not a
test.   python tools/skinny_ab.py [--reps 30] [--out gpurun_out/skinny_ab.jsonl]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import _lib  # noqa: E402
from onetrainer_amd import kernels as K  # noqa: E402

# (M tokens, N = fused rank, K): SDXL 1024^2 b=4 levels 2 / 3 (16384 / 4096 tokens), FLUX 768^2 b=4 (4 x 2381)
SHAPES = [(4096, 96, 1280), (4096, 32, 1280), (4096, 32, 5120), (4096, 64, 1280), (4096, 96, 3840), (4096, 32, 10240),
          (16384, 96, 640), (16384, 32, 640), (16384, 32, 2560), (16384, 96, 1920), (16384, 32, 5120),
          (9524, 48, 3072), (9524, 16, 3072), (9524, 16, 12288), (9524, 64, 3072)]


def timeit(fn, reps):
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
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/skinny_ab.jsonl")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.lib()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        for M, N, Kd in SHAPES:
            g = torch.Generator(device=dev).manual_seed(M + N + Kd)
            x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
            w = (torch.randn(N, Kd, device=dev, generator=g) * 0.05).bfloat16()
            ref = x.float() @ w.float().t()
            outs, times = {}, {0: [], 1: []}
            for on in (0, 1):
                lib.otamd_gemm_set_skinny(on)
                outs[on] = K.linear(x, w).float()
            for _ in range(a.rounds):
                for on in (0, 1):
                    lib.otamd_gemm_set_skinny(on)
                    K.linear(x, w)
                    times[on].append(timeit(lambda: K.linear(x, w), a.reps))
            lib.otamd_gemm_set_skinny(1)
            err = {on: ((outs[on] - ref).abs().max() / ref.abs().max()).item() for on in (0, 1)}
            t0, t1 = sorted(times[0])[a.rounds // 2], sorted(times[1])[a.rounds // 2]
            r = {"M": M, "N": N, "K": Kd, "us_split": round(t0, 2), "us_skinny": round(t1, 2), "speedup": round(t0 / t1, 3),
                 "GBps_skinny": round(M * Kd * 2 / t1 / 1e3, 1), "rel_err_split": round(err[0], 5),
                 "rel_err_skinny": round(err[1], 5)}
            print(json.dumps(r), flush=True)
            f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
