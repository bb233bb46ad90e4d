"""Time the fused AdamW(+SR) kernel on a 2.567 G-element bf16 store (SDXL UNet size): computed
denominator path vs LDS-table path (OTAMD_ADAMW_LUT), HIP-event average over 10 launches.

usage: python tools/adamw_probe.py [--n 2567000000]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import _lib, kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_567_000_000)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    n = a.n // 8 * 8
    dev = torch.device("cuda:0")
    p = (torch.randn(n, device=dev, dtype=torch.bfloat16) * 0.05)
    g = torch.randn(n, device=dev, dtype=torch.bfloat16) * 1e-3
    m = torch.zeros(n, device=dev, dtype=torch.bfloat16)
    v = torch.zeros(n, device=dev, dtype=torch.bfloat16)
    grp = [_lib.AdamwGroup(begin=0, end=n, wd_factor=1 - 1e-5, one_minus_beta1=0.1, beta2=0.999, one_minus_beta2=1e-3,
                           bc2_sqrt=0.0447, eps=1e-8, neg_step_size=-1e-3, pad=0.0)]
    for mode in ("0", "1", "2", "0", "1", "2"):
        os.environ["OTAMD_ADAMW_LUT"] = mode
        K.adamw_bf16(p, g, m, v, grp, stochastic_rounding=True, seed=1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.iters):
            K.adamw_bf16(p, g, m, v, grp, stochastic_rounding=True, seed=i)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        print(json.dumps({"lut": mode, "n": n, "ms": round(ms, 3), "TB_s": round(14 * n / ms / 1e9, 3)}), flush=True)
    # streaming roof: torch copy of 7 GB (read 3.5 + write 3.5 per element pair)
    del m, v
    a_ = torch.empty(n // 2 * 7 // 4, device=dev, dtype=torch.float32)
    b_ = torch.empty_like(a_)
    b_.copy_(a_)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        b_.copy_(a_)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    print(json.dumps({"copy_bytes": 2 * a_.numel() * 4, "ms": round(ms, 3), "TB_s": round(8 * a_.numel() / ms / 1e9, 3)}))


if __name__ == "__main__":
    main()
