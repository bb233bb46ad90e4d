"""The train loop with the step factored out: `train_step(batch)` has exactly
the semantics of the inlined step body at modules/trainer/GenericTrainer.py:672-749:

    predict -> calculate_loss -> / GA -> backward -> (update step: clip_grad_norm_ -> optimizer.step
    -> lr_scheduler.step -> zero_grad -> after_optimizer_step) -> train_progress.next_step

Differences, all MI355X-motivated and semantics-preserving:
  * no per-step host sync: the reference calls loss.item() every step (line 699); here the loss
    stays on device and is read every `log_every` steps;
  * the global clip runs on device and is applied inside the fused AdamW launch;
  * data parallel (new): gradient buckets are all-reduced from inside backward (trainer/ddp.py).
start()/train()/end() keep the reference's external behaviour (scripts/train.py:32-43).
"""
from __future__ import annotations

import time

import torch

from ..util import create
from ..util.lr_scheduler_util import create_lr_scheduler
from ..util.TrainProgress import TrainProgress
from .ddp import GradBucketReducer, init_from_env


class GenericTrainer:
    def __init__(self, config, callbacks=None, commands=None, model=None, model_setup=None, data_loader=None,
                 seed=0):
        self.config = config
        self.callbacks = callbacks
        self.commands = commands
        self.model = model
        self.model_setup = model_setup
        self.data_loader = data_loader
        self.seed = seed
        self.lr_scheduler = None
        self.reducer = None
        self.loss_history: list[torch.Tensor] = []

    # ------------------------------------------------------------------------------------------
    def start(self):
        cfg = self.config
        self.rank, self.world, local = init_from_env()
        self.device = torch.device(f"cuda:{local}") if torch.cuda.is_available() else torch.device(cfg.train_device)
        if self.model is None:
            self.model = create.create_model(cfg, self.device, seed=self.seed)
        if self.model_setup is None:
            self.model_setup = create.create_model_setup(cfg, self.device, self.rank, self.world)
        self.model_setup.setup_model(self.model, cfg)
        self.model_setup.setup_train_device(self.model, cfg)
        self.parameters = self.model.parameters.parameters()
        if self.world > 1:
            self.reducer = GradBucketReducer(self.model.train_store, bucket_bytes=cfg.dp_bucket_mb << 20)
        approx = self.data_loader.get_data_set().approximate_length() if self.data_loader is not None else 1
        self.lr_scheduler = create_lr_scheduler(self.model.optimizer, cfg.learning_rate_scheduler,
                                                cfg.learning_rate_warmup_steps, cfg.learning_rate_cycles,
                                                cfg.learning_rate_min_factor, cfg.epochs, approx,
                                                cfg.gradient_accumulation_steps,
                                                self.model.train_progress.global_step)

    def _is_update_step(self, tp: TrainProgress) -> bool:
        return (tp.global_step + 1) % self.config.gradient_accumulation_steps == 0

    def train_step(self, batch: dict) -> torch.Tensor:
        """one micro-step; returns the (device) loss divided by GA, like GenericTrainer.py:692."""
        cfg, model, setup = self.config, self.model, self.model_setup
        tp = model.train_progress
        store = model.train_store
        out = setup.predict(model, batch, cfg, tp)
        loss = setup.calculate_loss(model, batch, out, cfg)
        loss = loss / cfg.gradient_accumulation_steps
        store.begin_backward()
        loss.backward()
        store.finish_backward()
        if self._is_update_step(tp):
            if self.reducer is not None:
                self.reducer.finish()
            if cfg.clip_grad_norm is not None:
                model.optimizer.clip_grad_norm_(cfg.clip_grad_norm)
            model.optimizer.step()
            self.lr_scheduler.step()
            model.optimizer.zero_grad(set_to_none=True)
            setup.after_optimizer_step(model, cfg, tp)
        else:
            store.accumulating = True
        tp.next_step(cfg.batch_size)
        return loss.detach()

    def train(self, log_every: int = 10, max_steps: int | None = None):
        cfg = self.config
        tp = self.model.train_progress
        steps = 0
        for _epoch in range(tp.epoch, cfg.epochs):
            self.data_loader.get_data_set().start_next_epoch()
            for batch in self.data_loader.get_data_loader():
                loss = self.train_step(batch)
                self.loss_history.append(loss)
                steps += 1
                if log_every and steps % log_every == 0:
                    vals = torch.stack(self.loss_history[-log_every:]).float()
                    if self.world > 1:
                        torch.distributed.all_reduce(vals)
                        vals /= self.world
                    if self.rank == 0:
                        print(f"step {tp.global_step}: loss {vals.mean().item():.5f}", flush=True)
                if self.commands is not None and getattr(self.commands, "get_stop_command", lambda: False)():
                    return
                if max_steps is not None and steps >= max_steps:
                    return
            tp.next_epoch()

    def end(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
