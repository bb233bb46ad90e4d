"""VAE-encode (latent caching) throughput: SDXL AutoencoderKL encoder on synthetic [0,1] images,
resident in HBM.  Prints one JSON line (images/s, ms per batch, achieved TFLOP/s vs the bf16 peak).

usage: python tools/bench_vae.py [--res 1024 --batch 4 --iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd.module import vae as V  # noqa: E402


def run(res=1024, batch=4, iters=10, warmup=2, device="cuda:0"):
    dev = torch.device(device)
    enc = V.AutoencoderKLEncoder(V.sdxl_vae_config(), dev, seed=0)
    img = torch.rand(batch, 3, res, res, device=dev)
    for _ in range(warmup):
        enc.encode(img)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        lat = enc.encode(img)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    tf = V.flops_per_image(enc.cfg, res, res) * batch / (ms * 1e-3) / 1e12
    return {"what": "SDXL VAE encode (latent caching, mode=mean)", "res": res, "batch": batch,
            "images_per_s": round(batch / (ms * 1e-3), 2), "ms_per_batch": round(ms, 3),
            "achieved_tflops": round(tf, 1), "frac_bf16_peak": round(tf / 2500.0, 4),
            "latent_finite": bool(torch.isfinite(lat).all().item())}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    print(json.dumps(run(a.res, a.batch, a.iters)))
