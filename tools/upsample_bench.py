"""2x nearest-upsample backward (otamd_upsample2x_bwd) alone at the SDXL upsamplers' shapes (not a test): HIP-event
median per call, bytes / time, and a digest of the result (compare across library builds with OTAMD_LIB_ALT)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for N, H2, W2, C in [(4, 128, 128, 640), (4, 64, 64, 1280), (2, 96, 144, 320)]:
    dup = torch.randn(N, H2, W2, C, device=dev, generator=g).bfloat16()
    out = K.upsample2x_bwd(dup)
    acc = out.clone()
    K.upsample2x_bwd(dup, out=acc, accumulate=True)
    ts = []
    for _ in range(30):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        K.upsample2x_bwd(dup, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    us = sorted(ts)[15]
    dig = int(out.view(torch.int16).to(torch.int64).sum()) + 7 * int(acc.view(torch.int16).to(torch.int64).sum())
    print(json.dumps({"shape": [N, H2, W2, C], "us": round(us, 2), "GBps": round(dup.numel() * 2.5 / us / 1e3, 1),
                      "digest": dig}), flush=True)
