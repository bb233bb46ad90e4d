"""Is the SDXL step (1024^2, b=4) ever waiting for the host?  (not a test)

Runs the bench workload's steps back to back (as bench.py times them) in three modes, interleaved over rounds:
  * plain;
  * with a GPU spin kernel (torch.cuda._sleep) of ~L ms queued on the main stream before each step, so the host
    starts issuing every step L ms ahead of the GPU.
If the GPU never waits for the host, each step costs exactly L ms more with the spin; every millisecond less is a
host-induced bubble the lead absorbed.  The spin's own duration is timed with HIP events in isolation.

usage: python tools/host_bound_probe.py [--steps 8] [--rounds 2] [--lead-ms 10 30]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch  # noqa: E402
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer  # noqa: E402
from onetrainer_amd.util.config.TrainConfig import TrainConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--lead-ms", type=float, nargs="+", default=[10.0, 30.0])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = TrainConfig.default_values()
    cfg.batch_size = 4
    cfg.learning_rate = 3e-6
    cfg.learning_rate_warmup_steps = 0
    tr = GenericTrainer(cfg)
    tr.start()
    batch = synthetic_sdxl_batch(4, 1024, 1024, dev, seed=0)
    for _ in range(3):
        tr.train_step(batch)
    torch.cuda.synchronize()
    # spin calibration: cycles per ms of the sleep kernel
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(int(2e7))
    e1.record()
    e1.synchronize()
    cyc_per_ms = 2e7 / e0.elapsed_time(e1)
    spins = {}
    for lead in args.lead_ms:
        c = int(lead * cyc_per_ms)
        e0.record()
        for _ in range(5):
            torch.cuda._sleep(c)
        e1.record()
        e1.synchronize()
        spins[lead] = (c, e0.elapsed_time(e1) / 5)
    import gc
    gc.collect()
    gc.freeze()
    gc.disable()
    res = {k: [] for k in [0.0] + list(args.lead_ms)}
    for rnd in range(args.rounds):
        for lead in res:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                if lead:
                    torch.cuda._sleep(spins[lead][0])
                tr.train_step(batch)
            torch.cuda.synchronize()
            res[lead].append((time.perf_counter() - t0) * 1e3 / args.steps)
    base = min(res[0.0])
    print(f"plain step: {', '.join(f'{v:.2f}' for v in res[0.0])} ms", flush=True)
    for lead in args.lead_ms:
        spin_ms = spins[lead][1]
        best = min(res[lead])
        print(f"lead {lead:g} ms (spin measured {spin_ms:.2f} ms): step {', '.join(f'{v:.2f}' for v in res[lead])} ms; "
              f"step - spin = {best - spin_ms:.2f} ms vs plain {base:.2f} ms -> host bubbles absorbed "
              f"{base - (best - spin_ms):.2f} ms/step", flush=True)


if __name__ == "__main__":
    main()
