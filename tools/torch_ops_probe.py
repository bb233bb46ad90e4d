"""Which torch (aten) kernels does one train step still launch?  Runs one SDXL step (default 512^2 b=1; the op set
does not depend on the resolution) under a TorchDispatchMode that records every non-view aten op with a CUDA
output, with the op's shapes and the innermost call site in this repository (autograd-engine ops have none: they
are its gradient accumulations).  Not a test.

    python tools/torch_ops_probe.py [--res 512]
"""
import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from onetrainer_amd.dataLoader.SyntheticDataLoader import synthetic_sdxl_batch  # noqa: E402
from onetrainer_amd.module import unet as U  # noqa: E402
from onetrainer_amd.trainer.GenericTrainer import GenericTrainer  # noqa: E402
from onetrainer_amd.util import create  # noqa: E402
from onetrainer_amd.util.config.TrainConfig import TrainConfig  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKIP = {"empty", "empty_strided", "detach", "_to_copy_meta", "record_stream", "set_", "lift_fresh", "alias",
        "_local_scalar_dense", "is_same_size"}


class Probe(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func._schema.name.split("::")[-1]
        if getattr(func, "is_view", False) or name in SKIP:
            return out
        outs = out if isinstance(out, (tuple, list)) else (out,)
        if not any(torch.is_tensor(o) and o.is_cuda and o.numel() > 0 for o in outs):
            return out
        site = "autograd engine"
        for fr in reversed(traceback.extract_stack()[:-1]):
            if fr.filename.startswith(REPO) and "torch_ops_probe" not in fr.filename:
                site = f"{os.path.relpath(fr.filename, REPO)}:{fr.lineno}"
                break
        shapes = tuple(tuple(a.shape) for a in args if torch.is_tensor(a))
        self.ops[(name, shapes, site)] += 1
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=512)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = TrainConfig.default_values()
    cfg.batch_size = 1
    cfg.learning_rate_warmup_steps = 0
    model = create.create_model(cfg, dev, seed=0, unet_config=U.sdxl_config())
    tr = GenericTrainer(cfg, model=model)
    tr.start()
    batch = synthetic_sdxl_batch(1, a.res, a.res, dev, seed=0)
    tr.train_step(batch)
    torch.cuda.synchronize()
    with Probe() as p:
        tr.train_step(batch)
    torch.cuda.synchronize()
    total = sum(p.ops.values())
    print(f"{total} aten launches with CUDA outputs in one step")
    for (name, shapes, site), n in p.ops.most_common():
        print(f"{n:5d}  {name:28s} {site:45s} {shapes}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
