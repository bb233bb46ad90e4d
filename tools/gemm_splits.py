"""Split-K probe (not a test): for each (op, M, N, K) of the SDXL step's split-K GEMMs and each
forced split count, run the GEMM `reps` times; configurations are separated by a torch fill
kernel so that `tools/gemm_splits.py --db <rocprofv3 DB>` can attribute GEMM and split-K reduce
durations per configuration afterwards.

usage: rocprofv3 --kernel-trace -d gpurun_out/splits -o run -- python tools/gemm_splits.py
       python tools/gemm_splits.py --db gpurun_out/splits/run_results.db
"""
import argparse
import collections
import json
import os
import sqlite3
import sys

SHAPES = [  # (op, M, N, K) in GEMM terms
    ("dgrad", 4096, 1280, 10240),
    ("dgrad", 16384, 640, 5120),
    ("dgrad", 4096, 1280, 5120),
    ("wgrad", 1280, 1280, 4096),
    ("wgrad", 640, 640, 16384),
    ("wgrad", 1280, 5120, 4096),
    ("fwd", 4096, 1280, 5120),
]
SPLITS = [1, 2, 3, 4, 6, 8]


def run(reps):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from onetrainer_amd import kernels as K

    dev = torch.device("cuda:0")
    marker = torch.zeros(1, device=dev)
    for op, M, N, Kd in SHAPES:
        if op == "fwd":
            x = torch.randn(M, Kd, device=dev).bfloat16()
            w = torch.randn(N, Kd, device=dev).bfloat16()
        elif op == "dgrad":
            x = torch.randn(M, Kd, device=dev).bfloat16()     # dy [M, Nout=Kd]
            w = torch.randn(Kd, N, device=dev).bfloat16()     # w [Nout, Nin=N]
        else:
            dy = torch.randn(Kd, M, device=dev).bfloat16()
            xx = torch.randn(Kd, N, device=dev).bfloat16()
        for s in SPLITS:
            for _ in range(reps):
                if op == "fwd":
                    K._gemm_forced_splits = s
                    K.linear(x, w)
                elif op == "dgrad":
                    K._gemm_forced_splits = s
                    K.linear_dgrad(x, w)
                else:
                    K.linear_wgrad(dy, xx, splits=s)
            torch.cuda.synchronize()
            marker.fill_(float(s))
            torch.cuda.synchronize()
            print(json.dumps({"op": op, "M": M, "N": N, "K": Kd, "splits": s}), flush=True)
        K._gemm_forced_splits = 0


def analyse(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    groups, cur = [], collections.defaultdict(list)
    for name, s, e in rows:
        if "fill" in name.lower() and "gemm" not in name:
            groups.append(cur)
            cur = collections.defaultdict(list)
            continue
        if "gemm" in name or "splitk" in name:
            cur["reduce" if "splitk" in name else "gemm"].append((e - s) / 1e3)
    cfgs = [(op, M, N, Kd, s) for op, M, N, Kd in SHAPES for s in SPLITS]
    for cfg, g in zip(cfgs, groups[-len(cfgs):]):
        gm = sorted(g["gemm"])[len(g["gemm"]) // 2] if g["gemm"] else 0
        rd = sorted(g["reduce"])[len(g["reduce"]) // 2] if g["reduce"] else 0
        op, M, N, Kd, s = cfg
        print(json.dumps({"op": op, "M": M, "N": N, "K": Kd, "splits": s, "gemm_us": round(gm, 1),
                          "reduce_us": round(rd, 1), "total_us": round(gm + rd, 1),
                          "reduce_GBps": round((s * M * N * 4 + M * N * 2) / (rd * 1e-6) / 1e9, 0) if rd else None}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--db")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    if a.db:
        analyse(a.db)
    else:
        run(a.reps)
