"""Run train steps under the stream-ordering hazard checker (module/stream_hazards.py) and print what it finds.

    python tools/hazard_probe.py [--model sdxl|sd15|sdxl-lora] [--res 512] [--batch 1] [--steps 2]
exit status 1 when a hazard was found
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch  # noqa: E402
from onetrainer_amd.module.stream_hazards import StreamHazardCheck  # noqa: E402
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer  # noqa: E402
from onetrainer_amd.util.config.TrainConfig import TrainConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="sdxl", choices=["sdxl", "sd15", "sdxl-lora"])
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    cfg = TrainConfig.default_values()
    sd15 = a.model == "sd15"
    if sd15:
        cfg.model_type = "STABLE_DIFFUSION_15"
    if a.model == "sdxl-lora":
        cfg.training_method, cfg.lora_rank = "LORA", 32
    cfg.batch_size = a.batch
    cfg.learning_rate_warmup_steps = 0
    tr = GenericTrainer(cfg, seed=0)
    tr.start()
    batch = synthetic_sdxl_batch(a.batch, a.res, a.res, tr.device, seed=0, sdxl=not sd15,
                                 scaling_factor=0.18215 if sd15 else 0.13025)
    tr.train_step(batch)      # first sight of the shape outside the checker (plans, workspaces)
    torch.cuda.synchronize()
    with StreamHazardCheck() as chk:
        for _ in range(a.steps):
            tr.train_step(batch)
    torch.cuda.synchronize()
    print(chk.report(limit=60), flush=True)
    return 1 if chk.hazards else 0


if __name__ == "__main__":
    sys.exit(main())
