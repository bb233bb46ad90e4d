"""The train loop with the step factored out: `train_step(batch)` has exactly
the semantics of the inlined step body at modules/trainer/GenericTrainer.py:672-749:

    predict -> calculate_loss -> / GA -> backward -> (update step: clip_grad_norm_ -> optimizer.step
    -> lr_scheduler.step -> zero_grad -> after_optimizer_step) -> train_progress.next_step

Differences, all MI355X-motivated and semantics-preserving:
  * no per-step host sync: the reference calls loss.item() every step (line 699); here the loss
    stays on device and is read every `log_every` steps;
  * the global clip runs on device and is applied inside the fused AdamW launch;
  * data parallel (new): gradient buckets are all-reduced from inside backward (trainer/ddp.py);
  * single-GPU, opt-in (OTAMD_STEP_GRAPH=1): forward + backward captured once per batch shape and
    replayed as one HIP graph (trainer/step_graph.py; measured slower than the two-stream eager step).
start()/train()/end() keep the reference's external behaviour (scripts/train.py:32-43).
"""
from __future__ import annotations

import gc
import time

import torch

from ..util import create
from ..util.config.plain import plain
from ..util.lr_scheduler_util import create_lr_scheduler
from ..util.TimedActionMixin import TimedActionMixin
from ..util.TrainCommands import TrainCommands
from ..util.TrainProgress import TrainProgress
from .ddp import GradBucketReducer, abort, init_from_env


class GenericTrainer(TimedActionMixin):
    def __init__(self, config, callbacks=None, commands=None, model=None, model_setup=None, data_loader=None,
                 seed=0):
        super().__init__()
        self.config = plain(config)       # the reference's enum-typed TrainConfig or this build's
        self.callbacks = callbacks
        self.commands = commands if commands is not None else TrainCommands()
        self.model = model
        self.model_setup = model_setup
        self.data_loader = data_loader
        self.seed = seed
        self.lr_scheduler = None
        self.reducer = None
        self.graphs = None
        self.loss_history: list[torch.Tensor] = []
        self.tensorboard = None            # util/tensorboard.ScalarLog, opened by train()
        self._micro_losses: list[torch.Tensor] = []         # this update step's micro-step losses (device)
        self._update_losses: list[tuple[int, list[torch.Tensor]]] = []   # (global_step, losses) not yet logged
        self._ema_loss = None
        self._ema_loss_steps = 0
        self.one_step_trained = False
        self._has_gradient = False
        self._wallclock_timers = False
        self._det_flags = 0                # backup / save raised by STEP / EPOCH timers under DP (_raise_timed)
        self._ctl_group = None
        self.agreements = 0
        self.rank, self.world = 0, 1

    # ------------------------------------------------------------------------------------------
    def start(self):
        cfg = self.config
        self.rank, self.world, local = init_from_env()
        self.device = torch.device(f"cuda:{torch.cuda.current_device()}") if torch.cuda.is_available() \
            else torch.device(str(cfg.train_device))
        if self.model is None:
            self.model = create.create_model(cfg, self.device, seed=self.seed)
        from ..dataLoader.create import attach_cache_encoders, cache_ready, create_data_loader, has_concepts
        # create.create_data_loader (create.py:391-431) when there is data to load: a latent cache at
        # cache_dir or concepts to cache; step-level callers (bench, tests) pass batches to train_step
        want_data = self.data_loader is None and (cache_ready(cfg) or has_concepts(cfg))
        if want_data and not cache_ready(cfg):   # the model loader fills the caching encoders
            attach_cache_encoders(self.model, cfg, self.device)
        self._load_weights()
        if want_data:
            self.data_loader = create_data_loader(cfg, self.model, self.device, self.rank, self.world)
        if self.model_setup is None:
            self.model_setup = create.create_model_setup(cfg, self.device, self.rank, self.world)
        self.model_setup.setup_model(self.model, cfg)
        self.model_setup.setup_train_device(self.model, cfg)
        plan = getattr(self.model, "dtype_plan", None)
        if plan is not None and plan.overrides and self.rank == 0:   # util/dtype_util.py: recorded, not silent
            print(f"dtype policy: {plan.summary()}", flush=True)
        self.parameters = self.model.parameters.parameters()
        import os
        emulate = int(os.environ.get("OTAMD_DP_EMULATE", "0") or 0)
        if self.world > 1:
            self.reducer = GradBucketReducer(self.model.train_store, bucket_bytes=cfg.dp_bucket_mb << 20,
                                             reduce_fp32=cfg.dp_reduce_fp32)
        elif emulate > 1 and self.device.type == "cuda":   # RCCL's on-chip footprint at world N, on one GPU (ddp.py)
            self.reducer = GradBucketReducer(self.model.train_store, bucket_bytes=cfg.dp_bucket_mb << 20, emulate=emulate,
                                             emulate_blocks=int(os.environ.get("OTAMD_DP_EMULATE_CUS", "64")),
                                             emulate_gbs=float(os.environ.get("OTAMD_DP_EMULATE_GBS", "400")))
        approx = self.data_loader.get_data_set().approximate_length() if self.data_loader is not None else 1
        self.lr_scheduler = create_lr_scheduler(self.model.optimizer, cfg.learning_rate_scheduler,
                                                cfg.learning_rate_warmup_steps, cfg.learning_rate_cycles,
                                                cfg.learning_rate_min_factor, cfg.epochs, approx,
                                                cfg.gradient_accumulation_steps,
                                                self.model.train_progress.global_step)
        from .step_graph import StepGraphs
        if StepGraphs.enabled_for(self):
            self.graphs = StepGraphs(self)
        self._attach_norm_overlap()

    def _attach_norm_overlap(self):
        """eager steps, clip on, the fused AdamW: clip_grad_norm_'s norm pass runs during backward
        (util/optimizer/adamw_fused.OverlappedGradNorm) -- in one process as gradient ranges finish, under data
        parallel as the reducer's buckets finish their all-reduce (the norm of the global-mean gradients)."""
        import os

        from ..module import streams as S
        from ..util.optimizer.adamw_fused import FusedAdamW, OverlappedGradNorm
        opt = getattr(self.model, "optimizer", None)
        if (isinstance(opt, FusedAdamW) and self.graphs is None and self.config.clip_grad_norm
                and opt.store.grad.is_cuda and S.enabled() and os.environ.get("OTAMD_NORM_OVERLAP", "1") != "0"
                and opt.norm_overlap is None):
            opt.norm_overlap = OverlappedGradNorm(opt, reducer=self.reducer,
                                                  bucket_bytes=int(os.environ.get("OTAMD_NORM_BUCKET_MB", "64")) << 20)

    def _load_weights(self):
        """base / VAE / LoRA weights and a backup to continue from (GenericTrainer.py:92-108 +
        the model loader); with nothing named the model keeps its seeded random init."""
        cfg = self.config
        names = cfg.model_names()
        if cfg.continue_last_backup:
            last = cfg.get_last_backup_path()
            if last:
                if cfg.training_method == "LORA":
                    names.lora = last
                else:
                    names.base_model = last
                print(f"Continuing training from backup '{last}'...")
            else:
                print("No backup found, continuing without backup...")
        if names.base_model or names.lora:
            from ..modelLoader import create_model_loader
            create_model_loader(cfg.model_type, cfg.training_method).load(self.model, names)

    def backup(self, train_progress: TrainProgress | None = None) -> str | None:
        """INTERNAL backup to <workspace>/backup/<timestamp>-backup-<global_step>-<epoch>-<epoch_step>
        (GenericTrainer.py:406-449): model (diffusers layout / LoRA file), optimizer with
        param_group_mapping, meta.json, onetrainer_config/args.json; rank 0 writes, a failed backup is
        removed, rolling backups keep the newest `rolling_backup_count`."""
        import json
        import os
        import shutil
        import traceback
        from datetime import datetime

        from ..modelSaver import create_model_saver
        cfg = self.config
        tp = train_progress or self.model.train_progress
        if self.world > 1:
            torch.distributed.barrier()
        path = None
        if self.rank == 0:
            name = f"{datetime.now().strftime('%Y-%m-%d_%H-%M-%S')}-backup-{tp.filename_string()}"
            path = os.path.join(cfg.workspace_dir, "backup", name)
            try:
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
                create_model_saver(cfg.model_type, cfg.training_method).save(self.model, cfg, "INTERNAL", path)
                os.makedirs(os.path.join(path, "onetrainer_config"), exist_ok=True)
                with open(os.path.join(path, "onetrainer_config", "args.json"), "w") as f:
                    json.dump(cfg.to_settings_dict(), f, indent=4, default=str)
            except Exception:
                traceback.print_exc()
                print("Could not save backup. Check your disk space!")
                shutil.rmtree(path, ignore_errors=True)
                path = None
            finally:
                if cfg.rolling_backup:
                    self._prune_backups(cfg.rolling_backup_count)
        if self.world > 1:
            torch.distributed.barrier()
        return path

    def _prune_backups(self, keep: int):
        import os
        import shutil
        root = os.path.join(self.config.workspace_dir, "backup")
        if os.path.exists(root):
            dirs = sorted((d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d))), reverse=True)
            for d in dirs[keep:]:
                shutil.rmtree(os.path.join(root, d), ignore_errors=True)

    def save(self, train_progress: TrainProgress | None = None, print_msg: bool = True, print_cb=print) -> str | None:
        """periodic save (GenericTrainer.py:453-497) to <workspace>/save/<prefix><timestamp>-save-
        <global_step>-<epoch>-<epoch_step><ext> in output_model_format / output_dtype; rank 0 writes,
        a failed save is reported and its partial output removed."""
        import os
        from datetime import datetime
        cfg = self.config
        tp = train_progress or self.model.train_progress
        path = os.path.join(cfg.workspace_dir, "save",
                            f"{cfg.save_filename_prefix}{datetime.now().strftime('%Y-%m-%d_%H-%M-%S')}-save-"
                            f"{tp.filename_string()}{_file_extension(cfg.output_model_format)}")
        if print_msg and self.rank == 0:
            print_cb("Saving " + path)
        return self._write_model(path, cfg.output_model_format)

    def _write_model(self, path: str, fmt: str) -> str | None:
        import os
        import shutil
        import traceback

        from ..modelSaver import create_model_saver
        cfg = self.config
        ok = True
        if self.rank == 0:
            try:
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
                create_model_saver(cfg.model_type, cfg.training_method).save(self.model, cfg, fmt, path,
                                                                              _torch_dtype(cfg.output_dtype))
            except Exception:
                traceback.print_exc()
                print("Could not save model. Check your disk space!")
                ok = False
                if os.path.isdir(path):
                    shutil.rmtree(path, ignore_errors=True)
                elif os.path.isfile(path):
                    os.remove(path)
        if self.world > 1:
            torch.distributed.barrier()
        return path if ok else None

    def final_model_path(self) -> str:
        """end()'s destination (GenericTrainer.py:778-785): a single-file format into an existing
        directory gets a timestamped file name inside it."""
        import os
        from datetime import datetime
        cfg = self.config
        dest = cfg.output_model_destination
        ext = _file_extension(cfg.output_model_format)
        if os.path.isdir(dest) and ext:
            return os.path.join(dest, f"{cfg.save_filename_prefix}{datetime.now().strftime('%Y-%m-%d_%H-%M-%S')}{ext}")
        return dest

    def _is_update_step(self, tp: TrainProgress) -> bool:
        return (tp.global_step + 1) % self.config.gradient_accumulation_steps == 0

    def train_step(self, batch: dict) -> torch.Tensor:
        """one micro-step; returns the (device) loss divided by GA, like GenericTrainer.py:692."""
        cfg, model, setup = self.config, self.model, self.model_setup
        tp = model.train_progress
        store = model.train_store
        update = self._is_update_step(tp)
        if self.reducer is not None:   # GA micro-steps accumulate locally; the update step's backward reduces
            self.reducer.arm(update)
        norm = getattr(model.optimizer, "norm_overlap", None)
        loss = self.graphs.forward_backward(batch) if self.graphs is not None else None
        if loss is None:   # eager (or the first sight of a shape before its capture: trainer/step_graph.py)
            out = setup.predict(model, batch, cfg, tp)
            loss = setup.calculate_loss(model, batch, out, cfg)
            loss = loss / cfg.gradient_accumulation_steps
            store.begin_backward()
            if norm is not None:
                norm.arm(update and cfg.clip_grad_norm is not None)
            loss.backward()
            store.finish_backward()
            if norm is not None and not norm.dp:
                norm.finish()
        if update:
            if self.reducer is not None:
                self.reducer.finish()   # the last buckets, their norm sums (reduced_hooks), the post stream joined
                if norm is not None and norm.dp:
                    norm.finish()
            if cfg.clip_grad_norm is not None:
                model.optimizer.clip_grad_norm_(cfg.clip_grad_norm)
            model.optimizer.step()
            self.lr_scheduler.step()
            model.optimizer.zero_grad(set_to_none=True)
            if self.tensorboard is not None:   # GenericTrainer.py:720-722: lr/* at this update's global_step
                setup.report_to_tensorboard(model, cfg, self.lr_scheduler, self.tensorboard)
            setup.after_optimizer_step(model, cfg, tp)
            self.one_step_trained = True      # GenericTrainer.py:749: only after an optimizer update
        else:
            store.accumulating = True
        self._has_gradient = not update
        tp.next_step(cfg.batch_size)
        return loss.detach()

    # ----- the loop ----------------------------------------------------------------------------
    def _needs_backup(self, tp) -> bool:
        """GenericTrainer.py:506-509"""
        cfg = self.config
        return self.repeating_action_needed("backup", cfg.backup_after, cfg.backup_after_unit, tp, start_at_zero=False)

    def _needs_save(self, tp) -> bool:
        """GenericTrainer.py:511-516"""
        cfg = self.config
        return (self.single_action_elapsed("save_skip_first", cfg.save_skip_first, cfg.save_every_unit, tp)
                and self.repeating_action_needed("save", cfg.save_every, cfg.save_every_unit, tp, start_at_zero=False))

    agree_every = 16   # update steps between the ranks' backup / save agreements under wall-clock timers
    WALLCLOCK = ("SECOND", "MINUTE", "HOUR")

    def _agreement_point(self, tp) -> bool:
        """whether this (update-boundary) step consumes the sticky backup / save commands.  Always in one process
        or with only STEP / EPOCH timers; with a wall-clock timer under data parallel only every `agree_every`
        update steps, where rank 0's decision is broadcast (_agree), so the ranks do not meet on the host at every
        step.  Commands raised by a STEP / EPOCH timer under data parallel do not wait for this point (train():
        every rank raises them at the same step, so they run at the exact step, as in the reference)."""
        if self.world == 1 or not self._wallclock_timers:
            return True
        return (tp.global_step // self.config.gradient_accumulation_steps) % self.agree_every == 0

    def _raise_timed(self, kind: int, unit):
        """a timer fired before this step (GenericTrainer.py:653-656): a command the next update boundary runs.
        Under data parallel with wall-clock timers, STEP / EPOCH timers fire identically on every rank and are
        kept apart from the sticky commands that need rank 0's decision."""
        if self.world > 1 and self._wallclock_timers and TimedActionMixin._unit(unit) not in self.WALLCLOCK:
            self._det_flags |= kind
        elif kind == 1:
            self.commands.backup()
        else:
            self.commands.save()

    def _agree(self, flags: int, step: int) -> int:
        """Ranks must take a backup / save together (both barrier).  A wall-clock timer can fire on one
        rank and not another, so at an agreement point rank 0's flags are broadcast over a host-side gloo
        group (no device sync, no keys left in the rendezvous store) and every rank acts on them."""
        if self.world == 1 or not self._wallclock_timers:
            return flags
        import torch.distributed as dist
        if self._ctl_group is None:   # every rank reaches its first agreement point together
            self._ctl_group = dist.new_group(backend="gloo")
        t = torch.tensor([flags], dtype=torch.int64)
        dist.broadcast(t, src=0, group=self._ctl_group)
        self.agreements += 1
        return int(t.item())

    def train(self, log_every: int = 10, max_steps: int | None = None):
        """GenericTrainer.py:600-749 around train_step(): backup_after / save_every timers raise the
        backup / save commands before a step; the commands run at the next optimizer-update boundary
        (no accumulated gradient pending); stop is checked after every step and epoch."""
        cfg = self.config
        tp = self.model.train_progress
        if self.data_loader is None:
            raise RuntimeError("no data: set cache_dir to a latent cache or configure concepts")
        self._wallclock_timers = any(TimedActionMixin._unit(u) in ("SECOND", "MINUTE", "HOUR")
                                     for u in (cfg.backup_after_unit, cfg.save_every_unit))
        steps = 0
        # losses are read from the device every `flush_every` steps: printed when log_every is set, written as
        # the loss scalars either way (the reference logs them every update step, GenericTrainer.py:723-733)
        flush_every = log_every or 32
        self._det_flags = 0
        frozen = False
        failed = True
        if self.tensorboard is None:
            self.tensorboard = self._open_scalar_log()
        try:
            for _epoch in range(tp.epoch, cfg.epochs):
                self.data_loader.get_data_set().start_next_epoch()
                for batch in self.data_loader.get_data_loader():
                    if self._needs_backup(tp):
                        self._raise_timed(1, cfg.backup_after_unit)
                    if self._needs_save(tp):
                        self._raise_timed(2, cfg.save_every_unit)
                    if not self._has_gradient:
                        self._run_commands(tp, self._agreement_point(tp))
                    gs, update = tp.global_step, self._is_update_step(tp)
                    loss = self.train_step(batch)
                    self.loss_history.append(loss)
                    self._micro_losses.append(loss)
                    if update:   # GenericTrainer.py:723-733 (values resolved at the next flush point)
                        self._update_losses.append((gs, self._micro_losses))
                        self._micro_losses = []
                    steps += 1
                    if steps == 1:
                        # long-lived objects (model, plans, workspaces) out of the collector's generations; cyclic
                        # GC then runs only at the log points below, not as a pause inside a step's kernel issue
                        gc.collect()
                        gc.freeze()
                        gc.disable()
                        frozen = True
                    if steps % flush_every == 0:
                        gc.collect()
                        self._report_losses(flush_every, echo=bool(log_every))
                    if self.commands.get_stop_command() or (max_steps is not None and steps >= max_steps):
                        failed = False
                        return
                tp.next_epoch()
                if self.commands.get_stop_command():
                    failed = False
                    return
            failed = False
        finally:
            if failed and self.world > 1:
                self.abort_distributed()
            else:
                if not failed and steps % flush_every:
                    self._report_losses(steps % flush_every, echo=bool(log_every))   # the tail since the last flush
                if not failed and self.world > 1 and self._wallclock_timers and not self._has_gradient:
                    # a wall-clock command raised since the last agreement point: every rank ends the loop at the
                    # same step, so one more agreement here runs it instead of dropping it
                    self._run_commands(tp, True)
            if frozen:
                gc.unfreeze()
            gc.enable()

    def _run_commands(self, tp, agreement: bool):
        """at an update boundary (no accumulated gradient pending): the backup / save the timers or the command
        object asked for (GenericTrainer.py:653-668); sticky commands only at an agreement point"""
        flags, self._det_flags = self._det_flags, 0
        if agreement:
            sticky = (int(self.commands.get_and_reset_backup_command())
                      | int(self.commands.get_and_reset_save_command()) << 1)
            flags |= self._agree(sticky, tp.global_step)
        if flags & 1:
            self.backup(tp)
        if flags & 2:
            self.save(tp)

    def abort_distributed(self):
        """a rank failed (exception, timed-out collective, KeyboardInterrupt) inside train(): abort the
        process group so the rank exits instead of leaving peers blocked in a collective; the peers'
        own collectives time out (ddp.init_from_env) and abort the same way."""
        print(f"rank {self.rank}: training failed, aborting the process group", flush=True)
        self.reducer = None
        self.world = 1
        abort()

    def _open_scalar_log(self):
        """<workspace>/tensorboard/<prefix><timestamp> (GenericTrainer.py:66-68); rank 0 writes."""
        import os
        from datetime import datetime

        from ..util.tensorboard import ScalarLog
        cfg = self.config
        name = f"{cfg.save_filename_prefix}{datetime.now().strftime('%Y-%m-%d_%H-%M-%S')}"
        return ScalarLog(os.path.join(cfg.workspace_dir, "tensorboard", name), enabled=self.rank == 0)

    def _report_losses(self, n: int, echo: bool = True):
        """the log point: the mean of the last n micro-step losses printed, and per completed update step
        `loss/train_step` (the sum of its micro-step losses) and `smooth_loss/train_step` (the EMA with decay
        min(0.99, 1 - 1/k)) as GenericTrainer.py:722-732 computes them, all read in one device->host copy
        (averaged over ranks under data parallel)."""
        ups = self._update_losses
        flat = self.loss_history[-n:] + [l for _, ls in ups for l in ls]
        vals = torch.stack(flat).float()
        if self.world > 1:
            torch.distributed.all_reduce(vals)
            vals /= self.world
        host = vals.tolist()
        if self.rank == 0 and echo:
            print(f"step {self.model.train_progress.global_step}: loss {sum(host[:n]) / n:.5f} "
                  f"lr {self.lr_scheduler.get_last_lr()[0]:.3e}", flush=True)
        i = n
        tb = self.tensorboard
        for gs, ls in ups:
            acc = 0.0
            for v in host[i:i + len(ls)]:
                acc += v
            i += len(ls)
            self._ema_loss = self._ema_loss or acc
            self._ema_loss_steps += 1
            decay = min(0.99, 1 - (1 / self._ema_loss_steps))
            self._ema_loss = (self._ema_loss * decay) + (acc * (1 - decay))
            if tb is not None:
                tb.add_scalar("loss/train_step", acc, gs)
                tb.add_scalar("smooth_loss/train_step", self._ema_loss, gs)
        self._update_losses = []
        if tb is not None:
            tb.flush()
        del self.loss_history[:-n]

    def end(self):
        """GenericTrainer.py:766-806: after at least one trained step, a backup first when
        backup_before_save is set, then the final model to output_model_destination in
        output_model_format / output_dtype (rank 0 writes)."""
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if self.tensorboard is not None:
            self.tensorboard.close()
        if not self.one_step_trained:
            return None
        cfg = self.config
        if cfg.backup_before_save:
            self.backup(self.model.train_progress)
        path = self.final_model_path()
        if self.rank == 0:
            print("Saving " + path)
        return self._write_model(path, cfg.output_model_format)


def _file_extension(fmt: str) -> str:
    """ModelFormat.file_extension (modules/util/enum/ModelFormat.py)"""
    return {"CKPT": ".ckpt", "SAFETENSORS": ".safetensors", "LEGACY_SAFETENSORS": ".safetensors"}.get(str(fmt), "")


def _torch_dtype(name: str):
    """DataType.torch_dtype (modules/util/enum/DataType.py:19-36)"""
    return {"FLOAT_32": torch.float32, "TFLOAT_32": torch.float32, "BFLOAT_16": torch.bfloat16,
            "FLOAT_16": torch.float16}.get(str(name))
