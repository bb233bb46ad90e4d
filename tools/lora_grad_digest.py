"""Per-step digests of the SDXL LoRA adapter gradients (not a test): run the C4 train step a few times and print, per
step, the loss and a 64-bit digest of every adapter gradient tensor's bits, so two runs of this script can be diffed to
find the first step and tensor whose gradient is not bit-repeatable.

usage: python tools/lora_grad_digest.py [--steps 3] [--res 1024] [--batch 4]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch  # noqa: E402
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer  # noqa: E402
from onetrainer_amd.util.config.TrainConfig import TrainConfig  # noqa: E402


def digest(t: torch.Tensor) -> int:
    v = t.contiguous().view(torch.int32).to(torch.int64)
    w = torch.arange(1, v.numel() + 1, device=v.device, dtype=torch.int64) * 2654435761
    return int(((v * w) % (1 << 61)).sum().item() % (1 << 61))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--arb", action="store_true", help="one aspect bucket per step, as bench.py --model sdxl-lora")
    a = ap.parse_args()
    cfg = TrainConfig.default_values()
    cfg.training_method, cfg.lora_rank = "LORA", 32
    cfg.batch_size = a.batch
    cfg.learning_rate = 3e-4
    cfg.learning_rate_warmup_steps = 0
    tr = GenericTrainer(cfg, seed=0)
    tr.start()
    store = tr.model.train_store
    ov = getattr(tr.model.optimizer, "norm_overlap", None)
    if ov is not None and not ov.dp:   # the overlapped grad-norm ranges (backward order)
        for bi, (c0, c1, names) in enumerate(ov.buckets):
            n = sum(store.slots[x].numel for x in names)
            print(f"bucket {bi} chunks {c0}-{c1} numel {n} first {names[0]} last {names[-1]}")
    if a.arb:
        from onetrainer_amd.dataLoader.aspect_bucketing import ASPECTS, AspectBucketing
        buckets = AspectBucketing(a.res, 64, ASPECTS[:4]).resolutions
        batches = [synthetic_sdxl_batch(a.batch, r[0], r[1], tr.device, seed=0) for r in buckets]
    else:
        batches = [synthetic_sdxl_batch(a.batch, a.res, a.res, tr.device, seed=0)]
    for step in range(a.steps):
        loss = tr.train_step(batches[step % len(batches)])
        torch.cuda.synchronize()
        lv = float(loss) if loss is not None else float("nan")
        print(f"step {step} loss {lv!r} norm {float(tr.model.optimizer.clip_out[1])!r}", flush=True)
        for n in store.order:
            s = store.slots[n]
            print(f"  {step} {n} {digest(store.grad[s.offset:s.offset + s.numel])}")


if __name__ == "__main__":
    main()
