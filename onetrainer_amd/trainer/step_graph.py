"""Whole-step HIP graph for the train step's forward + backward (MI355X-first: graphs instead of a
tracing compiler; no reference counterpart -- the reference launches every op from Python).

OPT-IN (OTAMD_STEP_GRAPH=1).  The SDXL step issues ~4,000 kernels through autograd and the native host layer:
71-77 ms of host time per ~133 ms GPU step.  A captured step replays with ONE host call (37 ms of host issue per
step, round 4), but ran 145-147 ms on the GPU against 134 ms eager on the same box
(profiles/r4_step_graph_and_fork_order.txt): the GPU, not the host, bounds the step today, so the eager
two-stream step stays the default.

What is captured and what stays eager (GenericTrainer.train_step):
  eager   noise + timesteps (Philox, seeded by global_step) into static buffers
          (setup.step_inputs(..., out=...)); the batch copied into static buffers when the caller
          hands over other tensors
  graph   predict (DDPM prologue, UNet forward) -> MSE loss -> backward, including the weight-
          gradient side stream (module/streams.py: the side stream joins the capture through the
          event waits and is joined back by store.finish_backward)
  eager   clip_grad_norm_, fused AdamW, LR step, zero_grad (their scalars -- lr, bias corrections,
          SR seed -- change every step)
A shape (ARB bucket) runs eagerly the first time it is seen (GEMM plans, workspaces, LDS opt-ins
happen there) and is captured on its second occurrence; all graphs share one memory pool (they
never run concurrently).  Off when the step has host-varying inputs (text dropout masks), under
gradient accumulation (the first micro-step overwrites gradients, later ones accumulate), and with
data parallel (the bucket all-reduces are issued from inside backward; RCCL capture is not used).

Correctness.  Under the runtime's default graph execution the replayed step is bit-identical to the eager step
(tests/test_train_step_gpu.py::test_step_graph_matches_eager).  One round-4 run with the debug knob
DEBUG_HIP_FORCE_GRAPH_QUEUES=2 ended on another loss (1.0354 vs 0.90086; the same knob on another box matched).
Round 5 checked the two places such a race could come from: the captured graph has one root and one sink, with
the weight-gradient branch joined into finish_backward (tests/test_stream_hazards_gpu.py, from
hipGraphDebugDotPrint), and module/stream_hazards.StreamHazardCheck finds no main-stream access racing with the
side stream in the SDXL, SD 1.5 and LoRA steps, at the aten layer and at every kernel entry point (and does find
races planted on purpose).  The graph's edges therefore order every side-stream access the eager events order;
the outlier is attributed to the runtime's multi-queue execution under that debug knob, which is not used.
"""
from __future__ import annotations

import os

import torch


class _Entry:
    __slots__ = ("graph", "batch", "noise", "timestep", "loss")


class StepGraphs:
    def __init__(self, trainer):
        self.tr = trainer
        self.entries: dict = {}
        self.seen: dict = {}
        self.pool = None

    @staticmethod
    def enabled_for(trainer) -> bool:
        if os.environ.get("OTAMD_STEP_GRAPH", "0") != "1":
            return False
        setup, cfg = trainer.model_setup, trainer.config
        # an overlapped optimizer update orders the next forward through host-side waits (PRef.w ->
        # wait_params) that a replayed graph would skip: the two opt-ins are exclusive
        if getattr(trainer.model.optimizer, "overlap", False):
            return False
        return (trainer.device.type == "cuda" and trainer.world == 1 and trainer.reducer is None
                and cfg.gradient_accumulation_steps == 1 and hasattr(setup, "graphable")
                and hasattr(setup, "step_inputs") and setup.graphable(cfg))

    @staticmethod
    def _key(batch: dict) -> tuple:
        k = []
        for name in sorted(batch):
            v = batch[name]
            if torch.is_tensor(v):
                k.append((name, tuple(v.shape), v.dtype, str(v.device)))
            elif isinstance(v, (list, tuple)):
                k.append((name, tuple(str(x) for x in v)))
            else:
                k.append((name, repr(v)))
        return tuple(k)

    def _body(self, batch: dict) -> torch.Tensor:
        tr = self.tr
        cfg, model, setup = tr.config, tr.model, tr.model_setup
        out = setup.predict(model, batch, cfg, model.train_progress)
        loss = setup.calculate_loss(model, batch, out, cfg) / cfg.gradient_accumulation_steps
        store = model.train_store
        store.begin_backward()
        loss.backward()
        store.finish_backward()
        return loss.detach()

    debug_dot = None   # a path: capture in debug mode and write the graph's DOT there (tests, tools/graph_dump.py)

    def _capture(self, batch: dict) -> _Entry:
        tr = self.tr
        setup = tr.model_setup
        e = _Entry()
        e.batch = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in batch.items()}
        lat = e.batch["latent_image"]
        shape = tuple(setup._nhwc_latent(lat).shape)
        e.noise = torch.empty(shape, dtype=lat.dtype, device=lat.device)
        e.timestep = torch.empty(shape[0], dtype=torch.int32, device=lat.device)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()   # the eager steps' cached blocks; the graph gets its own pool
        g = torch.cuda.CUDAGraph(keep_graph=bool(self.debug_dot))   # debug: keep the hipGraph_t for the dump
        if self.debug_dot:
            g.enable_debug_mode()
        setup.graph_inputs = (e.noise, e.timestep)
        try:
            with torch.cuda.graph(g, pool=self.pool):
                e.loss = self._body(e.batch)
        finally:
            setup.graph_inputs = None
        if self.pool is None:
            self.pool = g.pool()
        if self.debug_dot:
            g.debug_dump(self.debug_dot)
        e.graph = g
        return e

    def forward_backward(self, batch: dict):
        """loss (a fresh tensor) after a replayed forward + backward, or None: run it eagerly."""
        key = self._key(batch)
        e = self.entries.get(key)
        if e is None:
            n = self.seen.get(key, 0)
            self.seen[key] = n + 1
            if n == 0:
                return None
            e = self.entries[key] = self._capture(batch)
        tr = self.tr
        for k, v in batch.items():
            if torch.is_tensor(v):
                dst = e.batch[k]
                if dst.data_ptr() != v.data_ptr():
                    dst.copy_(v, non_blocking=True)
        tr.model_setup.step_inputs(tr.model, e.batch, tr.config, tr.model.train_progress,
                                   out=(e.noise, e.timestep))
        e.graph.replay()
        return e.loss.clone()
