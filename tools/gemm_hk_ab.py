"""Same-process A/B of the two K-loop schedules of the v2 GEMM tiles (otamd_gemm_set_schedule: 0 = whole K-tile
DMA, gemm2_kernel.h; 1 = half-K DMA units, gemm2h_kernel.h) on the SDXL step's shapes and the large squares; not a
test.  Each (shape, plan) is timed with HIP events in interleaved rounds (median of the rounds' medians) and both
outputs are compared bit for bit (the two schedules sum the same products in the same order).

    python tools/gemm_hk_ab.py [--rounds 5] [--reps 30] [--out gpurun_out/gemm_hk_ab.jsonl]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import _lib  # noqa: E402
from onetrainer_amd import kernels as K  # noqa: E402

# (op, M, N, K, tile, splits): the main stream's largest 256- and 128-wide-tile GEMMs of the SDXL step (plans as the
# table picks them) and large squares
CASES_ALL = [
    ("fwd", 4096, 4096, 4096, 0, 1), ("fwd", 8192, 8192, 8192, 0, 1),
    ("dgrad", 4096, 1280, 10240, 0, 3), ("dgrad", 4096, 1280, 10240, 0, 1),
    ("fwd", 4096, 10240, 1280, 4, 1), ("fwd", 4096, 10240, 1280, 8, 1), ("fwd", 4096, 10240, 1280, 0, 1),
    ("fwd", 4096, 3840, 1280, 0, 1), ("dgrad", 4096, 5120, 1280, 8, 1), ("fwd", 4096, 1280, 5120, 7, 2),
    ("fwd", 4096, 1280, 1280, 4, 1), ("dgrad", 4096, 1280, 1280, 4, 1), ("fwd", 4096, 1280, 1280, 7, 1),
    ("fwd", 16384, 5120, 640, 0, 1), ("fwd", 16384, 640, 2560, 8, 1), ("dgrad", 16384, 640, 5120, 7, 1),
    ("wgrad", 10240, 1280, 4096, 0, 1), ("wgrad", 1280, 1280, 4096, 4, 2), ("wgrad", 3840, 1280, 4096, 7, 2),
    ("wgrad", 1280, 5120, 4096, 2, 1),
    # weight gradients with the bias gradient fused (column sums of dY), the step's own plans (None: plan table)
    ("wgrad_bias", 10240, 1280, 4096, None, 0), ("wgrad_bias", 1280, 1280, 4096, None, 0),
    ("wgrad_bias", 1280, 5120, 4096, None, 0), ("wgrad_bias", 640, 640, 16384, None, 0),
    # 3x3 conv weight gradients (+ bias): (N, H, W, Cin, Cout) in M / N / K
    ("convw_bias", 4, 32, 1280, None, 0), ("convw_bias", 4, 64, 640, None, 0), ("convw_bias", 4, 128, 320, None, 0),
]
CASES = CASES_ALL


def make(op, M, N, Kd, tile, splits, dev):
    g = torch.Generator(device=dev).manual_seed(M * 7 + N * 3 + Kd)
    BF = torch.bfloat16
    key_modes = {"fwd": (0, 0), "dgrad": (0, 1), "wgrad": (1, 1), "wgrad_bias": (1, 1), "convw_bias": (1, 4)}[op]
    if op == "fwd":
        x = torch.randn(M, Kd, device=dev, generator=g).to(BF)
        w = (torch.randn(N, Kd, device=dev, generator=g) * 0.05).to(BF)
        fn = lambda: K.linear(x, w)   # noqa: E731
    elif op == "dgrad":
        x = torch.randn(M, Kd, device=dev, generator=g).to(BF)
        w = (torch.randn(Kd, N, device=dev, generator=g) * 0.05).to(BF)
        fn = lambda: K.linear_dgrad(x, w)   # noqa: E731
    elif op == "wgrad":
        dy = torch.randn(Kd, M, device=dev, generator=g).to(BF)
        x = torch.randn(Kd, N, device=dev, generator=g).to(BF)
        out = torch.empty(M, N, device=dev, dtype=BF)
        fn = lambda: K.linear_wgrad(dy, x, out=out)   # noqa: E731
    elif op == "wgrad_bias":
        dy = torch.randn(Kd, M, device=dev, generator=g).to(BF)
        x = torch.randn(Kd, N, device=dev, generator=g).to(BF)
        out = torch.empty(M, N, device=dev, dtype=BF)
        bg = torch.empty(M, device=dev, dtype=BF)

        def fn():
            K.linear_wgrad(dy, x, out=out, bias_grad=bg)
            return out, bg
    else:   # convw_bias: M = batch, N = spatial side, Kd = channels (Cin = Cout)
        B, S, C_ = M, N, Kd
        x = torch.randn(B, S, S, C_, device=dev, generator=g).to(BF)
        dy = torch.randn(B, S, S, C_, device=dev, generator=g).to(BF)
        out = torch.empty(C_, 3, 3, C_, device=dev, dtype=BF)
        bg = torch.empty(C_, device=dev, dtype=BF)

        def fn():
            K.conv2d_wgrad(dy, x, 3, 1, 1, out=out, bias_grad=bg)
            return out, bg
        M, N, Kd = C_, 9 * C_, B * S * S
    return fn, key_modes + (M, N, Kd)


def timeit(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for i in range(reps):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))
    return ts[len(ts) // 2] * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--out", default="gpurun_out/gemm_hk_ab.jsonl")
    ap.add_argument("--ops", default=None, help="comma list: only these ops (fwd, dgrad, wgrad, wgrad_bias, convw_bias)")
    a = ap.parse_args()
    global CASES
    if a.ops:
        CASES = [c for c in CASES_ALL if c[0] in a.ops.split(",")]
    dev = torch.device("cuda:0")
    lib = _lib.lib()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        for op, M, N, Kd, tile, splits in CASES:
            fn, key = make(op, M, N, Kd, tile, splits, dev)
            os.environ["OTAMD_GEMM_PLAN"] = ",".join(map(str, key)) + f":{tile}:{splits}" if tile is not None else ""
            K._PLAN_OVERRIDES = None
            M, N, Kd = key[2:]
            outs, times = {}, {0: [], 1: []}
            for hk in (0, 1):
                lib.otamd_gemm_set_schedule(hk)
                o = fn()
                outs[hk] = [t.clone() for t in (o if isinstance(o, tuple) else (o,))]
                for _ in range(3):
                    fn()
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for hk in (0, 1):
                    lib.otamd_gemm_set_schedule(hk)
                    times[hk].append(timeit(fn, a.reps))
            lib.otamd_gemm_set_schedule(0)
            fl = 2.0 * M * N * Kd
            t0, t1 = sorted(times[0])[a.rounds // 2], sorted(times[1])[a.rounds // 2]
            r = {"op": op, "M": M, "N": N, "K": Kd, "tile": tile, "splits": splits, "us_base": round(t0, 2),
                 "us_hk": round(t1, 2), "tf_base": round(fl / t0 / 1e6, 1), "tf_hk": round(fl / t1 / 1e6, 1),
                 "speedup": round(t0 / t1, 3), "bitwise_equal": all(torch.equal(x, y) for x, y in zip(outs[0], outs[1]))}
            print(json.dumps(r), flush=True)
            f.write(json.dumps(r) + "\n")
            del outs
    return 0


if __name__ == "__main__":
    sys.exit(main())
