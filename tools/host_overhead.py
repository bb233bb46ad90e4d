"""Host issue time vs GPU time of the SDXL train step (1024^2, b=4): for each step, the time the
Python host needs to enqueue the whole step (no sync) and the step's wall time to completion.
HO_LORA=<rank>: the LoRA step (C4: r32); HO_PROFILE=1: cProfile of one step."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch  # noqa: E402
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer  # noqa: E402
from onetrainer_amd.util import create  # noqa: E402
from onetrainer_amd.util.config.TrainConfig import TrainConfig  # noqa: E402

dev = torch.device("cuda:0")
cfg = TrainConfig.default_values()
cfg.batch_size = int(os.environ.get("HO_BATCH", "4"))
if int(os.environ.get("HO_LORA", "0")):
    cfg.training_method, cfg.lora_rank = "LORA", int(os.environ["HO_LORA"])
model = create.create_model(cfg, dev, seed=0)
tr = GenericTrainer(cfg, model=model)
tr.start()
res = int(os.environ.get("HO_RES", "1024"))
batch = synthetic_sdxl_batch(cfg.batch_size, res, res, dev, seed=0)
for _ in range(3):
    tr.train_step(batch)
torch.cuda.synchronize()
for i in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train_step(batch)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"step {i}: host issue {1e3 * (t1 - t0):.1f} ms, wall {1e3 * (t2 - t0):.1f} ms", flush=True)
if os.environ.get("HO_PROFILE", "0") == "1":   # where the host issue time goes (cProfile, one step)
    import cProfile
    import pstats
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    with torch.autograd.set_multithreading_enabled(False):   # backward's Python on this thread (profiled)
        pr.enable()
        tr.train_step(batch)
        pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(45)
