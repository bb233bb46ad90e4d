"""Per-tile cost model probe: time Y = X W^T at M=N=4096 (240..256 tiles = one round) over K, for the
tile forced by OTAMD_GEMM_TILE; the slope is the main-loop cost per 64-deep K-step and the
intercept the fixed prologue/epilogue cost.  Prints one JSON line per K."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402


def timeit(fn, n=20):
    """GPU time per call: n calls captured in one graph and replayed (no host launch overhead)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


dev = torch.device("cuda:0")
M = int(os.environ.get("KSCAN_M", os.environ.get("KSCAN_MN", "4096")))
N = int(os.environ.get("KSCAN_N", os.environ.get("KSCAN_MN", "4096")))
for k in (64, 128, 256, 640, 1280, 2560, 5120, 10240):
    x = torch.randn(M, k, device=dev).bfloat16()
    w = torch.randn(N, k, device=dev).bfloat16()
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: K.linear(x, w, out=y))
    print(json.dumps({"tile": os.environ.get("OTAMD_GEMM_TILE", "plan"), "M": M, "N": N, "K": k, "us": round(t * 1e6, 2),
                      "tflops": round(2.0 * M * N * k / t / 1e12, 1)}), flush=True)
