"""Stream-ordering hazard checker (race detection: "stream-ordering asserts").

The step runs on two HIP streams (module/streams.py): every weight-gradient region hands tensors (dy, x,
LoRA t / u, LayerNorm statistics, the cross-attention dK / dV) to the side stream, ordered after the main
stream by a fork event, and the main stream waits for the side stream only at the join (finish_backward).
`record_stream` keeps the caching allocator from recycling such a tensor's block early, but nothing stops
the main stream from WRITING into that memory before the join -- and autograd does exactly that when it
accumulates two gradient contributions in place (`InputBuffer::accumulate`: `old.add_(new)` when it holds
the last reference).  Such a write races with the side stream's read: the weight gradient then sees
`dy + other` or `dy` depending on timing, which a replayed HIP graph (trainer/step_graph.py) shifts.

    with StreamHazardCheck() as chk:     # debug / test use only (TorchDispatchMode: slow)
        trainer.train_step(batch)
    assert not chk.hazards, chk.report()

Every aten op that writes a tensor (schema `(a!)` arguments, out= included) while the current stream is
not the side stream is checked against the byte ranges the side stream may still read; a hit is recorded
with the op, the tensor's shape and the region that handed the range over.  The HIP kernels themselves
write fresh outputs or the gradient store (on the side stream), so the aten layer is where a main-stream
write into a handed-over tensor can come from.
"""
from __future__ import annotations

import torch
from torch.utils._python_dispatch import TorchDispatchMode

from . import streams as S


def _span(t: torch.Tensor):
    """[lo, hi) bytes of the memory a strided tensor touches"""
    if t.numel() == 0 or not t.is_cuda:
        return None
    lo = t.data_ptr()
    ext = 1 + sum((n - 1) * abs(s) for n, s in zip(t.shape, t.stride()))
    return lo, lo + ext * t.element_size()


class StreamHazardCheck(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.pending: list = []     # (lo, hi, label): ranges the side stream may still read
        self.hazards: list = []
        self.regions = 0
        self.checked = 0

    # ---- hooks called from module/streams.py ------------------------------------------------------------
    def side_read(self, tensors, label: str):
        self.regions += 1
        for t in tensors:
            if torch.is_tensor(t):
                sp = _span(t)
                if sp is not None:
                    self.pending.append((sp[0], sp[1], label, tuple(t.shape)))

    def joined(self):
        self.pending.clear()

    # ---- the mode -----------------------------------------------------------------------------------------
    def __enter__(self):
        S._HAZARD.append(self)
        return super().__enter__()

    def __exit__(self, *exc):
        S._HAZARD.remove(self)
        return super().__exit__(*exc)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if self.pending:
            side = S.side_stream()
            cur = torch.cuda.current_stream()
            if side is None or cur.cuda_stream != side.cuda_stream:
                for i, a in enumerate(func._schema.arguments):
                    if a.alias_info is None or not a.alias_info.is_write:
                        continue
                    t = args[i] if i < len(args) else kwargs.get(a.name)
                    ts = t if isinstance(t, (list, tuple)) else (t,)
                    for x in ts:
                        if torch.is_tensor(x):
                            self._check(func, x)
        return func(*args, **kwargs)

    def _check(self, func, t):
        sp = _span(t)
        if sp is None:
            return
        self.checked += 1
        lo, hi = sp
        for plo, phi, label, shape in self.pending:
            if lo < phi and plo < hi:
                self.hazards.append((str(func), tuple(t.shape), label, shape))
                return

    def report(self, limit: int = 20) -> str:
        lines = [f"{len(self.hazards)} main-stream writes into memory the weight-gradient stream may still read "
                 f"({self.regions} side regions, {self.checked} writes checked)"]
        for op, shape, label, pshape in self.hazards[:limit]:
            lines.append(f"  {op} writes {list(shape)} over {label} input {list(pshape)}")
        return "\n".join(lines)
