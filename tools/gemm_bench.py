"""GEMM engine microbenchmark over the SDXL 1024^2 b=4 train-step shapes (not a test).

For every (op, M, N, K) the HIP kernel is timed with HIP events (median of reps) and compared with
torch.matmul (hipBLASLt) on the same operands as a yardstick.  Prints TFLOP/s per shape.
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from onetrainer_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
BF = torch.bfloat16


def timeit(fn, reps=20):
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
    return ts[len(ts) // 2] * 1e-3


SHAPES = [  # (name, M, N, K) of Y[M,N] = X[M,K] W[N,K]^T
    ("l1_qkv", 16384, 1920, 640), ("l1_out", 16384, 640, 640), ("l1_ff1", 16384, 5120, 640),
    ("l1_ff2", 16384, 640, 2560), ("l2_qkv", 4096, 3840, 1280), ("l2_out", 4096, 1280, 1280),
    ("l2_ff1", 4096, 10240, 1280), ("l2_ff2", 4096, 1280, 5120), ("kv_ctx", 308, 2560, 2048),
    ("big", 8192, 8192, 8192),
]
CONVS = [  # (name, N, H, W, Cin, Cout)
    ("c0", 4, 128, 128, 320, 320), ("c1", 4, 64, 64, 640, 640), ("c2", 4, 32, 32, 1280, 1280),
    ("c2cat", 4, 32, 32, 2560, 1280),
]

res = []
for name, M, N, Kd in SHAPES:
    x = torch.randn(M, Kd, device=dev).to(BF)
    w = (torch.randn(N, Kd, device=dev) * 0.05).to(BF)
    dy = torch.randn(M, N, device=dev).to(BF)
    dw = torch.empty(N, Kd, device=dev, dtype=BF)
    fl = 2.0 * M * N * Kd
    r = {"name": name, "M": M, "N": N, "K": Kd}
    r["fwd"] = fl / timeit(lambda: K.linear(x, w)) / 1e12
    r["dgrad"] = fl / timeit(lambda: K.linear_dgrad(dy, w)) / 1e12
    r["wgrad"] = fl / timeit(lambda: K.linear_wgrad(dy, x, out=dw)) / 1e12
    r["torch_fwd"] = fl / timeit(lambda: x @ w.t()) / 1e12
    r["torch_wgrad"] = fl / timeit(lambda: dy.t() @ x) / 1e12
    res.append(r)
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
for name, N, H, W, Ci, Co in CONVS:
    x = torch.randn(N, H, W, Ci, device=dev).to(BF)
    w = (torch.randn(Co, 3, 3, Ci, device=dev) * 0.02).to(BF)
    dy = torch.randn(N, H, W, Co, device=dev).to(BF)
    fl = 2.0 * N * H * W * Ci * Co * 9
    r = {"name": name, "shape": [N, H, W, Ci, Co]}
    r["fwd"] = fl / timeit(lambda: K.conv2d(x, w)) / 1e12
    r["dgrad"] = fl / timeit(lambda: K.conv2d_dgrad(dy, w, (H, W))) / 1e12
    r["wgrad"] = fl / timeit(lambda: K.conv2d_wgrad(dy, x, out=torch.empty_like(w))) / 1e12
    xn = x.permute(0, 3, 1, 2)
    wn = w.permute(0, 3, 1, 2)
    xc = xn.contiguous(memory_format=torch.channels_last)
    wc = wn.contiguous(memory_format=torch.channels_last)
    r["torch_fwd"] = fl / timeit(lambda: torch.nn.functional.conv2d(xc, wc, padding=1)) / 1e12
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
