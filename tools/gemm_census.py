"""GEMM census of one SDXL (1024^2, b=4) or FLUX.1 LoRA (768^2, b=4) train step: every GEMM/conv launch timed on the GPU with
events around it (includes the split-K reduce), grouped by (A mode, B mode, M, N, K, tile, splits).
Prints one JSON line per group, sorted by total time, plus the total.

usage: python tools/gemm_census.py [--steps 2]
"""
import argparse
import collections
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd import _lib, kernels as K  # noqa: E402
from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch  # noqa: E402
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer  # noqa: E402
from onetrainer_amd.util import create  # noqa: E402
from onetrainer_amd.util.config.TrainConfig import TrainConfig  # noqa: E402

MODES = {0: "K", 1: "MN", 2: "CONVF", 3: "CONVD", 4: "CONVW", 5: "WT"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--lora", type=int, default=0, help="LoRA rank (0: full fine-tune)")
    ap.add_argument("--flux", action="store_true", help="FLUX.1 LoRA r16 (C5) at --res (default 768)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = TrainConfig.default_values()
    cfg.batch_size = args.batch
    if args.lora:
        cfg.training_method, cfg.lora_rank = "LORA", args.lora
    if args.flux:
        cfg.model_type, cfg.training_method, cfg.timestep_distribution = "FLUX_DEV_1", "LORA", "LOGIT_NORMAL"
        if args.res == 1024:
            args.res = 768
    tr = GenericTrainer(cfg) if args.flux else GenericTrainer(cfg, model=create.create_model(cfg, dev, seed=0))
    tr.start()
    if args.flux:
        from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_flux_batch
        batch = synthetic_flux_batch(args.batch, args.res, args.res, dev, seed=0)
    else:
        batch = synthetic_sdxl_batch(args.batch, args.res, args.res, dev, seed=0)
    tr.train_step(batch)
    torch.cuda.synchronize()

    recs = []
    main_handle = torch.cuda.current_stream().cuda_stream
    K._HOST["off"] = True   # launch through the ctypes path, whose _gemm is wrapped below
    orig = K._gemm

    def timed(a, splits, device):
        s_out = C.c_int(0)
        _lib.lib().otamd_gemm_plan(C.byref(a), splits, C.byref(s_out))
        tile = _lib.lib().otamd_gemm_plan_tile(C.byref(a), splits)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(a, splits, device)
        e1.record()
        side = torch.cuda.current_stream().cuda_stream != main_handle
        key = (MODES[a.amode], MODES[a.bmode], a.M, a.N, a.K, tile, s_out.value, "side" if side else "main")
        recs.append((key, e0, e1))

    K._gemm = timed
    for _ in range(args.steps):
        tr.train_step(batch)
    torch.cuda.synchronize()
    K._gemm = orig
    agg = collections.defaultdict(lambda: [0, 0.0])
    for key, e0, e1 in recs:
        agg[key][0] += 1
        agg[key][1] += e0.elapsed_time(e1)
    total = 0.0
    for key, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        am, bm, M, N, Kd, tile, sp, st = key
        per = ms / args.steps
        total += per
        us = ms / n * 1e3
        print(json.dumps({"stream": st, "a": am, "b": bm, "M": M, "N": N, "K": Kd, "tile": tile, "splits": sp,
                          "calls_per_step": n / args.steps, "ms_per_step": round(per, 3), "us": round(us, 1),
                          "tflops": round(2.0 * M * N * Kd / (us * 1e-6) / 1e12, 1)}), flush=True)
    print(json.dumps({"total_ms_per_step": round(total, 2), "launches_per_step": len(recs) / args.steps}))


if __name__ == "__main__":
    main()
