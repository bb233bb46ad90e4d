"""Data-parallel gradient reduction over the flat gradient store (NEW: the reference has no DP,
SURVEY.md §2.4).  One process per GPU; torch.distributed 'nccl' is RCCL over xGMI on ROCm
('gloo' on CPU hosts for tests).

Buckets are contiguous slices of the flat grad buffer, formed in reverse layout order (the
store is laid out in forward-execution order, so reverse order ~ the order backward finishes
parameters).  Backward kernels write a parameter's gradient in place and call
`store.mark_ready`; when every parameter of a bucket is ready its all-reduce is issued with
async_op=True -- ProcessGroupNCCL orders it after the kernels already queued on the current
stream and runs it on its own stream, overlapping the rest of backward.  `finish()` makes the
current stream wait for all buckets.  The 1/world factor is folded into the loss gradient
(BaseStableDiffusionXLSetup.calculate_loss), so a SUM all-reduce yields the global-batch mean.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..module.streams import after_side


class GradBucketReducer:
    def __init__(self, store, group=None, bucket_bytes: int = 256 << 20):
        self.store = store
        self.group = group
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
        self.works = []
        self.enabled = True
        store.ready_hooks.append(self._on_ready)

    def _on_ready(self, names):
        if not self.enabled:
            return
        for n in names:
            bi = self.bucket_of[n]
            self.pending[bi] -= 1
            if self.pending[bi] == 0:
                b, e, _ = self.buckets[bi]
                g = self.store.grad[b:e]
                # ordered after both the main stream and the weight-gradient stream (module/streams.py)
                self.works.append(after_side(lambda: dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group,
                                                                     async_op=True)))

    def finish(self):
        """reduce any bucket not yet launched (unused params), then wait for all of them."""
        for bi, cnt in enumerate(self.pending):
            if cnt > 0:
                b, e, _ = self.buckets[bi]
                g = self.store.grad[b:e]
                self.works.append(after_side(lambda: dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group,
                                                                     async_op=True)))
        for w in self.works:
            w.wait()
        self.works = []
        self.pending = [len(b[2]) for b in self.buckets]


def init_from_env(backend: str | None = None):
    """torchrun-style env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT)."""
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local
