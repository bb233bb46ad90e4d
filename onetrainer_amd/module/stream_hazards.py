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

Two layers are checked, each against the byte ranges the side stream may still read or write (until the
next join):
  * every aten op (TorchDispatchMode): its written tensors (schema `(a!)` arguments, out= included) and
    read tensors while the current stream is not the side stream;
  * every HIP-kernel entry point of onetrainer_amd.kernels (wrapped while the checker is active): tensors
    named as outputs (returned, `out=`, `dx=`, `dq=` ... or an output parameter such as layernorm_param_grad's
    dgamma / dbeta) are writes, every other tensor argument a read.  A launch on the side stream adds its
    ranges to the pending sets; a launch on any other stream is checked: write vs pending read or write
    (WAR / WAW), read vs pending write (RAW).
A hit is recorded with the op, the tensor's shape and the call site that handed the range over.
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


# outputs of the kernels.py entry points besides their return values (keyword or positional parameter names)
_OUT_NAMES = {"out", "dx", "dq", "dk", "dv", "dgamma", "dbeta", "dmod", "dh", "grad_out", "bias_grad", "dw",
              "chunk_sq", "tensor_sq"}
_OUT_EXTRA = {"gated_add_bwd": {"dy"}, "adamw_bf16": {"p", "m", "v"}, "adamw_f32": {"p", "m", "v"},
              "softmax_rows_fwd": {"P", "lse"}, "softmax_rows_bwd": {"dS"}}
_NOT_KERNELS = {"stream_handle", "workspace", "set_gemm_autotune", "gemm_autotune_cache", "plan_source",
                "dump_plan_table", "host_layer", "pick_splits", "conv_out_hw", "python_host"}


def _tensors(v):
    if torch.is_tensor(v):
        yield v
    elif isinstance(v, (list, tuple)):
        for x in v:
            yield from _tensors(x)


class StreamHazardCheck(TorchDispatchMode):
    def __init__(self, kernels: bool = True):
        super().__init__()
        self.pending: list = []     # (lo, hi, label, shape): ranges the side stream may still read
        self.pending_w: list = []   # ... or still write
        self.hazards: list = []
        self.regions = 0
        self.checked = 0
        self.kernel_calls = 0
        self.allocated: set = set()   # storages allocated while the checker was active
        self.covered: set = set()     # storages record_stream()ed (to the side stream: the only one used)
        self.side_used: dict = {}     # storage -> (op, shape) used by side-stream kernels since the last join
        self._kernels = kernels
        self._saved = {}

    # ---- hooks called from module/streams.py ------------------------------------------------------------
    def side_read(self, tensors, label: str):
        self.regions += 1
        self._add(self.pending, tensors, label)

    @staticmethod
    def _add(lst, tensors, label):
        for t in _tensors(tensors):
            sp = _span(t)
            if sp is not None:
                lst.append((sp[0], sp[1], label, tuple(t.shape)))

    def joined(self):
        for st, (op, shape) in self.side_used.items():   # record_stream may come after the launch, before the free
            if st in self.allocated and st not in self.covered:
                self.hazards.append((op, "uses on the side stream", shape, "tensor never record_stream()ed", op, shape))
        self.side_used.clear()
        self.pending.clear()
        self.pending_w.clear()

    # ---- the mode -----------------------------------------------------------------------------------------
    def __enter__(self):
        S._HAZARD.append(self)
        if self._kernels:
            self._wrap_kernels()
        return super().__enter__()

    def __exit__(self, *exc):
        S._HAZARD.remove(self)
        from .. import kernels as K
        for name, fn in self._saved.items():
            setattr(K, name, fn)
        self._saved.clear()
        return super().__exit__(*exc)

    _NO_DATA = ("record_stream",)   # schema-marked mutations that touch no tensor data

    def _on_side(self) -> bool:
        side = S.side_stream()
        return side is not None and torch.cuda.current_stream().cuda_stream == side.cuda_stream

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = func._schema.name.split("::")[-1]
        if name == "record_stream":   # the allocator now defers this block's reuse until the side stream is done
            for t in _tensors(args[:1]):
                self.covered.add(t.untyped_storage().data_ptr())
            return func(*args, **kwargs)
        view = getattr(func, "is_view", False)
        if (self.pending or self.pending_w) and not view and not self._on_side():
            for i, a in enumerate(func._schema.arguments):
                t = args[i] if i < len(args) else kwargs.get(a.name)
                write = a.alias_info is not None and a.alias_info.is_write
                for x in _tensors(t):
                    self._check(str(func), x, write)
        out = func(*args, **kwargs)
        if not view and not any(r.alias_info is not None for r in func._schema.returns):
            for t in _tensors(out):   # a fresh block: the allocator handed it out, so whatever the side stream did
                self._fresh(t)        # with that memory before has completed (record_stream) -- or was never covered
        return out

    def _fresh(self, t):
        sp = _span(t)
        if sp is None:
            return
        if self._on_side():   # allocated on the side stream: its reuse is ordered by that stream, nothing to record
            self.covered.add(t.untyped_storage().data_ptr())
        self.allocated.add(t.untyped_storage().data_ptr())
        lo, hi = sp
        self.pending = [p for p in self.pending if not (lo < p[1] and p[0] < hi)]
        self.pending_w = [p for p in self.pending_w if not (lo < p[1] and p[0] < hi)]

    def _check(self, op, t, write: bool):
        sp = _span(t)
        if sp is None:
            return
        self.checked += 1
        lo, hi = sp
        for lst, kind in ((self.pending, "read"), (self.pending_w, "write")) if write else ((self.pending_w, "write"),):
            for plo, phi, label, shape in lst:
                if lo < phi and plo < hi:
                    self.hazards.append((op, "writes" if write else "reads", tuple(t.shape), kind, label, shape))
                    return

    def _side_use(self, op, t):
        """a tensor allocated during the checked region and used by the side stream must be record_stream()ed
        before it is freed (checked at the join)"""
        self.side_used.setdefault(t.untyped_storage().data_ptr(), (op, tuple(t.shape)))

    # ---- the kernels.py layer -----------------------------------------------------------------------------
    def _wrap_kernels(self):
        import inspect
        import sys
        from .. import kernels as K
        for name, fn in list(vars(K).items()):
            if name.startswith("_") or name in _NOT_KERNELS or not inspect.isfunction(fn) or fn.__module__ != K.__name__:
                continue
            try:
                sig = inspect.signature(fn)
            except (TypeError, ValueError):
                continue
            outs = _OUT_NAMES | _OUT_EXTRA.get(name, set())

            def wrapper(*args, __fn=fn, __sig=sig, __name=name, __outs=outs, **kwargs):
                try:
                    bound = __sig.bind(*args, **kwargs)
                except TypeError:
                    return __fn(*args, **kwargs)
                reads, writes, side_writes = [], [], []
                cast_side = __name == "attn_bwd" and bound.arguments.get("cast_stream") is not None
                for pname, v in bound.arguments.items():
                    if cast_side and pname in ("dk", "dv"):
                        side_writes.extend(_tensors(v))      # written on cast_stream (the side stream)
                    elif pname in __outs:
                        writes.extend(_tensors(v))
                    else:
                        reads.extend(_tensors(v))
                on_side = self._on_side()
                site = sys._getframe(1)
                label = f"{__name} from {site.f_code.co_filename.rsplit('/', 1)[-1]}:{site.f_lineno}"
                if not on_side:
                    for t in reads:
                        self._check(f"K.{__name}", t, False)
                    for t in writes:
                        self._check(f"K.{__name}", t, True)
                out = __fn(*args, **kwargs)
                self.kernel_calls += 1
                if on_side:
                    for t in reads + writes:
                        self._side_use(f"K.{__name}", t)
                    self._add(self.pending, reads, label)
                    self._add(self.pending_w, writes + list(_tensors(out)), label)
                else:
                    for t in side_writes:
                        self._side_use(f"K.{__name}", t)
                    self._add(self.pending_w, side_writes, label)
                return out

            self._saved[name] = fn
            setattr(K, name, wrapper)

    def report(self, limit: int = 20) -> str:
        import collections
        lines = [f"{len(self.hazards)} accesses that race with the weight-gradient stream "
                 f"({self.regions} side regions, {self.kernel_calls} kernel calls, {self.checked} accesses checked)"]
        kinds = collections.Counter((h[0], h[1], h[3], h[4]) for h in self.hazards)
        for (op, how, kind, label), n in kinds.most_common(limit):
            ex = next(h for h in self.hazards if (h[0], h[1], h[3], h[4]) == (op, how, kind, label))
            lines.append(f"  {n:5d} x {op} {how} {list(ex[2])} over a pending side-stream {kind} {list(ex[5])} ({label})")
        return "\n".join(lines)
