"""Run one attention shape a few times (PMC passes: tools/gpu_attn_pmc.sh).  Not a test.
usage: python tools/attn_one.py B Nq Nk H D [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import kernels as K  # noqa: E402

B, Nq, Nk, H, D = (int(x) for x in sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
dev = torch.device("cuda:0")
q = torch.randn(B, Nq, H * D, device=dev).to(torch.bfloat16)
k = torch.randn(B, Nk, H * D, device=dev).to(torch.bfloat16)
v = torch.randn(B, Nk, H * D, device=dev).to(torch.bfloat16)
do = torch.randn(B, Nq, H * D, device=dev).to(torch.bfloat16)
for _ in range(reps):
    o, lse = K.attn_fwd(q, k, v, H)
    K.attn_bwd(q, k, v, o, lse, do, H)
torch.cuda.synchronize()
