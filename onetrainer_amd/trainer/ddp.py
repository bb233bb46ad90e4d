"""Data-parallel gradient reduction over the flat gradient store (NEW: the reference has no DP,
SURVEY.md §2.4).  One process per GPU; torch.distributed 'nccl' is RCCL over xGMI on ROCm
('gloo' on CPU hosts for tests).

Buckets are contiguous slices of the flat grad buffer, formed in reverse layout order (the
store is laid out in forward-execution order, so reverse order ~ the order backward finishes
parameters).  Backward kernels write a parameter's gradient in place and call
`store.mark_ready`; when every parameter of a bucket is ready its all-reduce is issued with
async_op=True from a dedicated issue stream that waits (by events) on BOTH the compute stream
and the weight-gradient side stream (module/streams.py) -- neither compute stream is made to wait
for the other or for the collective, so the reduce overlaps the rest of backward.  `finish()`
makes the current stream wait for all buckets.  The 1/world factor is folded into the loss
gradient (BaseStableDiffusionXLSetup.calculate_loss), so a SUM all-reduce yields the
global-batch mean.

Gradient accumulation: the reducer is armed only for the backward of an update step
(`arm(update)` before every backward).  Earlier micro-steps accumulate locally into the grad
store; the last micro-step's backward launches each bucket once, over the accumulated sum.

Emulation (emulate=N, OTAMD_DP_EMULATE=N in GenericTrainer at world size 1): each bucket's all-reduce is replaced
by its on-chip footprint on this GPU -- a kernel on the issue stream, at the bucket's ready point, holding
`emulate_blocks` workgroups (RCCL's channels) for the ring's wire time 2 (N-1)/N S / busbw and moving as many
bytes through HBM (kernels.dp_emulate) -- so the slowdown RCCL's kernels cause the two compute streams is measured
on one GPU.  Gradients are left as they are.

Completion: on a GPU every bucket's completion is taken on a post stream -- it waits for the collective, copies an
fp32-staged bucket back, then runs `reduced_hooks(bucket)` (the clip norm's squared sums of the bucket's chunks,
util/optimizer/adamw_fused.OverlappedGradNorm), so clip_grad_norm_ after the last bucket only folds per-chunk sums
instead of re-reading every gradient (~1.8 ms per SDXL step); `finish()` orders the current stream after it.

Reduction dtype: bf16 in place (default: 2 B/param on the wire, the reference's grad dtype) or,
with `reduce_fp32=True`, through an fp32 staging copy (4 B/param; one rounding to bf16 after the
sum instead of one per ring hop).  tests/test_dp_gpu.py characterises both against a world-1
step at the same global batch.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..module import streams as S


class _EmulatedWork:
    """the async-work handle of an emulated bucket: wait() orders the current stream after the issue stream"""

    def __init__(self, stream):
        self.stream = stream

    def wait(self):
        torch.cuda.current_stream().wait_stream(self.stream)


class GradBucketReducer:
    def __init__(self, store, group=None, bucket_bytes: int = 256 << 20, reduce_fp32: bool = False, emulate: int = 0,
                 emulate_blocks: int = 64, emulate_gbs: float = 400.0):
        self.emulate, self.emulate_blocks, self.emulate_gbs = emulate, emulate_blocks, emulate_gbs
        self.scratch = None
        self.store = store
        self.group = group
        self.reduce_fp32 = reduce_fp32
        esz = store.grad.element_size()
        limit = max(1, bucket_bytes // esz)
        self.buckets = []         # (begin, end, names)
        cur, cur_begin, cur_end = [], None, None
        for name in reversed(store.order):
            s = store.slots[name]
            if cur and (cur_end - s.offset) > limit:
                self.buckets.append((cur_begin, cur_end, cur))
                cur = []
            if not cur:
                cur_end = s.offset + s.numel
                cur_end = (cur_end + 7) // 8 * 8
            cur.append(name)
            cur_begin = s.offset
        if cur:
            self.buckets.append((cur_begin, cur_end, cur))
        self.bucket_of = {}
        for bi, (_, _, names) in enumerate(self.buckets):
            for n in names:
                self.bucket_of[n] = bi
        self.pending = [len(b[2]) for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.works = []           # (work, bucket index)
        self.enabled = True
        self.staging = None       # fp32 copy of the flat grad buffer (reduce_fp32)
        cuda = store.grad.is_cuda
        self.issue_stream = torch.cuda.Stream(device=store.grad.device) if cuda else None
        # completion side: waits for each bucket's collective, copies a staged bucket back, runs reduced_hooks
        self.post_stream = torch.cuda.Stream(device=store.grad.device) if cuda else None
        self.reduced_hooks = []   # callables(bucket index), on post_stream once the bucket holds the global sum
        store.ready_hooks.append(self._on_ready)

    def arm(self, update_step: bool):
        """before each backward: only an update step's backward reduces (GA micro-steps accumulate)."""
        self.enabled = update_step
        self.pending = [len(b[2]) for b in self.buckets]
        self.launched = [False] * len(self.buckets)

    def _launch(self, bi):
        b, e, _ = self.buckets[bi]
        g = self.store.grad[b:e]
        self.launched[bi] = True
        if self.issue_stream is None:
            self.works.append((self._reduce(g, b, e), bi))
            return
        s = self.issue_stream
        # the deferred reduces write into this bucket: the side stream's split-K ones and this stream's LayerNorm
        # parameter ones (module/streams.py), flushed before the wait below orders the collective after them
        S.defer_flush()
        s.wait_stream(torch.cuda.current_stream())
        side = S.side_stream()
        if side is not None:
            s.wait_stream(side)
        with torch.cuda.stream(s):
            work = self._reduce(g, b, e)
        self.works.append((work, bi))
        with torch.cuda.stream(self.post_stream):
            work.wait()                        # stream-ordered for RCCL: this stream waits for the collective
            if self.reduce_fp32 and self.emulate <= 1:
                g.copy_(self.staging[b:e])     # the sum, rounded once to bf16
            for h in self.reduced_hooks:
                h(bi)

    def _reduce(self, g, b, e):
        if self.emulate > 1:
            from .. import kernels as K
            n = self.emulate
            wire = 2.0 * (n - 1) / n * g.numel() * g.element_size()
            if self.scratch is None:
                self.scratch = torch.empty(max(be - bb for bb, be, _ in self.buckets) * g.element_size(),
                                           dtype=torch.uint8, device=g.device)
            K.dp_emulate(g, self.scratch, int(wire) // 16 * 16, self.emulate_blocks, int(wire / self.emulate_gbs))
            return _EmulatedWork(torch.cuda.current_stream())
        if not self.reduce_fp32:
            return dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        if self.staging is None:
            self.staging = torch.empty(self.store.grad.numel(), dtype=torch.float32, device=g.device)
        buf = self.staging[b:e]
        buf.copy_(g)
        return dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def _on_ready(self, names):
        if not self.enabled:
            return
        for n in names:
            bi = self.bucket_of[n]
            self.pending[bi] -= 1
            if self.pending[bi] == 0 and not self.launched[bi]:
                self._launch(bi)

    def finish(self):
        """reduce any bucket not yet launched (parameters without a gradient this step), then make
        the current stream wait for every bucket."""
        for bi in range(len(self.buckets)):
            if not self.launched[bi]:
                self._launch(bi)
        if self.post_stream is not None:   # every bucket's completion went through the post stream (_launch)
            torch.cuda.current_stream().wait_stream(self.post_stream)
        else:
            for w, bi in self.works:
                w.wait()
                if self.reduce_fp32:
                    b, e, _ = self.buckets[bi]
                    self.store.grad[b:e].copy_(self.staging[b:e])
                for h in self.reduced_hooks:
                    h(bi)
        self.works = []
        self.arm(True)


DEFAULT_TIMEOUT_S = 600


def init_from_env(backend: str | None = None, timeout_s: float | None = None):
    """torchrun-style env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT).

    Failure detection: every collective of the group carries a timeout
    (OTAMD_DIST_TIMEOUT_S, default 600 s) -- a rank that died or hangs makes its peers' next
    collective raise instead of blocking forever -- and RCCL runs with asynchronous error handling
    (TORCH_NCCL_ASYNC_ERROR_HANDLING=1 unless set: the watchdog tears the communicator down on a
    timed-out or failed collective).  The trainer then aborts the group and the rank exits with the
    error (GenericTrainer.abort_distributed)."""
    import datetime
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("OTAMD_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if timeout_s is None:
            timeout_s = float(os.environ.get("OTAMD_DIST_TIMEOUT_S", DEFAULT_TIMEOUT_S))
        if backend == "nccl":
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        if torch.cuda.is_available():
            torch.cuda.set_device(local if backend == "nccl" else local % max(1, torch.cuda.device_count()))
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s))
    return rank, world, local


def abort():
    """tear the process group down after a failure so this rank can exit (no further collective is
    attempted; a peer blocked in one times out on its own)."""
    if dist.is_available() and dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:   # a broken communicator may refuse a clean shutdown; exiting is what matters
            pass
