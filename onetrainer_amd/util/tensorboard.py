"""Scalar log of the train loop (the reference's `SummaryWriter`, modules/trainer/GenericTrainer.py:66-68,
720-733): `add_scalar(tag, value, step)` with the same tags (`loss/train_step`, `smooth_loss/train_step`,
`lr/<group>`).

torch.utils.tensorboard needs the `tensorboard` package, which this image lacks: scalars are written as
JSON lines to `<log_dir>/scalars.jsonl` ({"tag", "value", "step", "wall_time"}), and to a SummaryWriter as
well when one imports.  Values may be device tensors: they stay on the device until flush(), which reads
them all with one copy, so logging adds no host sync to a step."""
from __future__ import annotations

import json
import os
import time

import torch


class ScalarLog:
    def __init__(self, log_dir: str, enabled: bool = True):
        self.log_dir = log_dir
        self.enabled = enabled
        self.pending: list[tuple[str, object, int, float]] = []
        self._writer = None
        self._file = None

    def _open(self):   # on the first flush with something to write: a run that logs nothing leaves no files
        os.makedirs(self.log_dir, exist_ok=True)
        self._file = open(os.path.join(self.log_dir, "scalars.jsonl"), "a")
        try:
            from torch.utils.tensorboard import SummaryWriter
            self._writer = SummaryWriter(self.log_dir)
        except Exception:   # tensorboard not installed: the JSON lines are the log
            self._writer = None

    def add_scalar(self, tag: str, value, step: int):
        if self.enabled:
            self.pending.append((tag, value, int(step), time.time()))

    def flush(self):
        if not self.enabled or not self.pending:
            return
        if self._file is None:
            self._open()
        dev = [v for _, v, _, _ in self.pending if torch.is_tensor(v)]
        host = iter(torch.stack([v.detach().float().reshape(()) for v in dev]).tolist()) if dev else iter(())
        for tag, v, step, wall in self.pending:
            val = next(host) if torch.is_tensor(v) else float(v)
            self._file.write(json.dumps({"tag": tag, "value": val, "step": step, "wall_time": wall}) + "\n")
            if self._writer is not None:
                self._writer.add_scalar(tag, val, step, walltime=wall)
        self.pending.clear()
        self._file.flush()
        if self._writer is not None:
            self._writer.flush()

    def close(self):
        self.flush()
        if self._file is not None:
            self._file.close()
            self._file = None
        if self._writer is not None:
            self._writer.close()
            self._writer = None


def read_scalars(log_dir: str) -> list[dict]:
    with open(os.path.join(log_dir, "scalars.jsonl")) as f:
        return [json.loads(line) for line in f if line.strip()]
