"""Flat parameter / gradient store.

All trainable tensors of a model live as views of ONE flat buffer (params) with a twin flat
buffer for gradients, each tensor at a 16-byte aligned offset.  Consequences:
  * the fused AdamW (csrc/adamw.hip) is a single pass over the flat buffers (14 B/param bf16);
  * data-parallel gradient buckets are contiguous slices of the flat grad buffer (trainer/ddp.py);
  * weights that one GEMM consumes together (to_q|to_k|to_v, to_k|to_v) are adjacent, so the
    fused projection weight and its gradient are plain views -- no concat, no split.
Backward kernels write weight gradients straight into `grad` views (overwrite on the first
micro-step of an accumulation window, accumulate afterwards) and call `mark_ready`, which feeds
the DP reducer; autograd never materialises or accumulates parameter gradients.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass
class Slot:
    name: str
    shape: tuple
    offset: int
    numel: int
    group: str


class FlatParamStore:
    def __init__(self, specs, dtype, device, align_bytes=16, trainable=True, master=False):
        """specs: iterable of (name, shape, group) in layout order.  trainable=False: a frozen base
        (LoRA training, unet.requires_grad_(False) in StableDiffusionXLLoRASetup.py:78-86): no grad
        buffer, parameters do not require grad, backward kernels skip its weight gradients.
        master=True: fp32 master weights (weight_dtype FLOAT_32, TrainConfig.py:782) behind the bf16 working copy
        `data` the kernels read -- `master` holds the trained values, `data` their round-to-nearest bf16 cast (what
        autocast feeds every GEMM, dtype_util.py:28-49); gradients stay bf16 (autocast's weight gradients are bf16
        GEMM results cast to fp32, so bf16 holds them exactly)."""
        esz = torch.tensor([], dtype=dtype).element_size()
        al = max(8, align_bytes // esz)   # >= 8 elements: the grad-norm kernel reads 8-wide chunks
        self.dtype, self.device = dtype, device
        self.slots: dict[str, Slot] = {}
        self.order: list[str] = []
        off = 0
        for name, shape, group in specs:
            n = 1
            for s in shape:
                n *= int(s)
            off = (off + al - 1) // al * al
            self.slots[name] = Slot(name, tuple(int(s) for s in shape), off, n, group)
            self.order.append(name)
            off += n
        self.numel = (off + al - 1) // al * al
        self.trainable = trainable
        self.data = torch.zeros(self.numel, dtype=dtype, device=device)
        if master and (not trainable or dtype != torch.bfloat16):
            raise ValueError("fp32 master weights back a trainable bf16 store")
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=device) if master else None
        self.grad = torch.zeros(self.numel, dtype=dtype, device=device) if trainable else None
        self._params: dict[str, torch.nn.Parameter] = {}
        for name in self.order:
            s = self.slots[name]
            p = torch.nn.Parameter(self.data[s.offset:s.offset + s.numel].view(s.shape), requires_grad=trainable)
            if trainable:
                p.grad = self.grad[s.offset:s.offset + s.numel].view(s.shape)
            self._params[name] = p
        self._written: set[str] = set()
        self.accumulating = False          # True on micro-steps after the first of a GA window
        self.ready_hooks = []              # callables(names) -> None (DP reducer)
        # optimizer update in flight on another stream (util/optimizer/adamw_fused.py): [(end element,
        # event)] in layout order; a consumer of element range [.., end) waits for the events up to it
        self.update_events: list | None = None
        self._waited = 0

    # ----- views -------------------------------------------------------------------------------
    @property
    def params(self) -> dict:
        """name -> parameter view.  A reader that takes weights from here (or from view()) rather than
        through PRef.w is ordered after an optimizer update still in flight on its own stream
        (util/optimizer/adamw_fused.py overlap): it waits for every pending chunk."""
        if self.update_events is not None:
            self.wait_params()
        return self._params

    def view(self, names, shape=None, grad=False):
        """contiguous view spanning `names` (which must be adjacent without padding); a weight view
        waits for the optimizer chunks covering it when an update is in flight."""
        if isinstance(names, str):
            names = [names]
        first = self.slots[names[0]]
        end = first.offset
        for n in names:
            s = self.slots[n]
            if s.offset != end:
                raise ValueError(f"parameters {names} are not adjacent in the flat store")
            end += s.numel
        buf = self.grad if grad else self.data
        if buf is None:
            return None
        if not grad and self.update_events is not None:
            self.wait_params(end)
        v = buf[first.offset:end]
        if shape is not None:
            v = v.view(shape)
        elif len(names) == 1:
            v = v.view(first.shape)
        return v

    def value(self, name):
        """the trained value of one tensor (store layout): the fp32 master view, else the parameter view."""
        s = self.slots[name]
        if self.master is not None:
            return self.master[s.offset:s.offset + s.numel].view(s.shape)
        return self.params[name].detach()

    @torch.no_grad()
    def write(self, name, value):
        """set one tensor (store layout); with master weights the fp32 value goes to the master and the working
        copy takes its bf16 cast."""
        s = self.slots[name]
        if self.master is not None:
            self.wait_params()
            mv = self.master[s.offset:s.offset + s.numel].view(s.shape)
            mv.copy_(value)
            self.data[s.offset:s.offset + s.numel].view(s.shape).copy_(mv)
        else:
            self.params[name].copy_(value)

    def range_of(self, names):
        first = self.slots[names[0]]
        last = self.slots[names[-1]]
        return first.offset, last.offset + last.numel

    # ----- asynchronous optimizer updates ------------------------------------------------------------
    def set_update_events(self, events):
        self.update_events = events or None
        self._waited = 0

    def wait_params(self, end: int | None = None):
        """make the current stream wait for the optimizer chunks covering elements [0, end) (all when
        end is None).  Forward order = layout order, so a forward that reaches layer L waits only for the
        chunks up to L's weights; the rest of the update keeps running beside it."""
        ev = self.update_events
        if ev is None:
            return
        cur = torch.cuda.current_stream(self.device)
        while self._waited < len(ev):
            e_end, e = ev[self._waited]
            cur.wait_event(e)
            self._waited += 1
            if end is not None and e_end >= end:
                break
        if self._waited >= len(ev):
            self.update_events = None

    # ----- gradient bookkeeping -----------------------------------------------------------------
    def accumulate_into(self, names) -> bool:
        """True if a backward kernel must add into the grad view (GA window), else overwrite."""
        return self.accumulating

    def mark_ready(self, names):
        self._written.update(names)
        for h in self.ready_hooks:
            h(names)

    def begin_backward(self):
        self.wait_params()   # backward overwrites the gradients the optimizer chunks read
        self._written.clear()
        if self.device.type == "cuda":
            from .streams import defer_begin
            defer_begin(self.grad if self.trainable else None)   # the gradient GEMMs' split-K reduces go out grouped

    def finish_backward(self):
        """join the weight-gradient stream, then zero the grads of parameters that received none
        this micro-step (overwrite semantics)."""
        if self.device.type == "cuda":
            from .streams import defer_end, join
            defer_end()      # the pending grouped split-K reduces, before anything reads the gradients
            join()
        if self.trainable and not self.accumulating:
            for n in self.order:
                if n not in self._written:
                    s = self.slots[n]
                    self.grad[s.offset:s.offset + s.numel].zero_()

    def named_parameters(self):
        return [(n, self._params[n]) for n in self.order]

    def group_ranges(self):
        """{group: (begin, end)} element ranges; groups must be contiguous in layout order."""
        out = {}
        for n in self.order:
            s = self.slots[n]
            b, e = out.get(s.group, (s.offset, s.offset + s.numel))
            out[s.group] = (min(b, s.offset), max(e, s.offset + s.numel))
        return out
