"""Side HIP stream for weight-gradient work (MI355X-first scheduling, no reference counterpart).

In backward every Linear / conv needs dgrad (on the critical path: the next layer's backward
waits for it) and wgrad + bias colsum (needed only by the optimizer / DP all-reduce).  At b = 4
many of these GEMMs fill only part of the 256 CUs (e.g. 4096 x 1280 x 1280: 160 tiles of
256 x 128), so running the weight-gradient GEMMs on a second stream lets them occupy the CUs the
dgrad chain leaves idle instead of serialising behind it.

    with wgrad_region(tensors):   # side stream waits for everything queued on the main stream so
        ...launch wgrad...        # far (dy, x ready), kernels go to the side stream; the tensors
                                  # are record_stream()ed so the caching allocator cannot recycle
                                  # them before the side stream has read them
    join()                        # main stream waits for the side stream (before clip / AdamW)

OTAMD_WGRAD_STREAM=0 disables it (everything on the current stream).  The GEMM workspace is
per stream (kernels.workspace), so the two streams never share split-K slabs.
"""
from __future__ import annotations

import os

import torch

_SIDE: dict = {}
_ENABLED = os.environ.get("OTAMD_WGRAD_STREAM", "1") != "0"


_AVAIL = None
_STREAMS: dict = {}   # raw HIP stream -> torch Stream object (current_stream() builds a new one per call)
_EVENTS: dict = {}    # side stream index -> reusable fork event (a wait captures the record current at enqueue)
_HAZARD: list = []    # active module/stream_hazards.StreamHazardCheck instances (debug / tests only)


def enabled() -> bool:
    global _AVAIL
    if _AVAIL is None:
        _AVAIL = torch.cuda.is_available()
    return _ENABLED and _AVAIL


def _current(idx: int):
    raw = torch._C._cuda_getCurrentRawStream(idx)
    st = _STREAMS.get(raw)
    if st is None:
        st = _STREAMS[raw] = torch.cuda.current_stream(idx)
    return st


def set_enabled(on: bool):
    global _ENABLED
    _ENABLED = bool(on)


_get_device = torch._C._cuda_getDevice


def side_stream(device=None):
    if not (_ENABLED and (_AVAIL if _AVAIL is not None else enabled())):
        return None
    idx = _get_device() if device is None else torch.device(device).index
    if idx is None:
        idx = _get_device()
    s = _SIDE.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _SIDE[idx] = s
    return s


class wgrad_region:
    """with wgrad_region(tensors): ... -- the enclosed launches go to the side stream, ordered after the main stream's
    work so far; the tensors are record_stream()ed to it on exit.  (A plain class: ~1,200 regions per SDXL step, and
    a generator-based context manager cost ~2 us of host time each.)"""
    __slots__ = ("tensors", "side", "main")

    def __init__(self, tensors=()):
        self.tensors = tensors

    def __enter__(self):
        side = self.side = side_stream()
        if side is None:
            return self
        idx = side.device_index
        main = self.main = _current(idx)
        ev = _EVENTS.get(idx)
        if ev is None:
            ev = _EVENTS[idx] = torch.cuda.Event()
        ev.record(main)
        side.wait_event(ev)
        torch.cuda.set_stream(side)
        return self

    def __exit__(self, *exc):
        side = self.side
        if side is None:
            return False
        torch.cuda.set_stream(self.main)
        if exc[0] is not None:
            return False
        for t in self.tensors:
            if t is not None and t.is_cuda:
                t.record_stream(side)
        if _HAZARD:
            note_side(self.tensors, 2)
        return False


def note_side(tensors, depth: int = 1):
    """tell an active hazard checker that the side stream may read these tensors until the next join()"""
    if _HAZARD:
        import sys
        fr = sys._getframe(depth)
        label = f"{fr.f_code.co_filename.rsplit('/', 1)[-1]}:{fr.f_lineno}"
        for h in _HAZARD:
            h.side_read(tensors, label)


_DEFER = os.environ.get("OTAMD_DEFER_REDUCE", "1") != "0"
_LN_DEFER = os.environ.get("OTAMD_LN_DEFER", "1") != "0"
_LN_STREAM: list = []   # the stream whose LayerNorm parameter reduces are deferred (kernels.ln_defer_begin)


def defer_begin(grads):
    """start of a backward: the side stream's split-K reduces into the flat gradient buffer `grads` are deferred and
    launched grouped (kernels.defer_reduces_begin; OTAMD_DEFER_REDUCE=0 launches each with its GEMM), and so are the
    current stream's LayerNorm dgamma / dbeta reduces (kernels.ln_defer_begin; OTAMD_LN_DEFER=0 launches each with
    its LayerNorm)"""
    if grads is None or not grads.numel():
        return
    from .. import kernels as K
    side = side_stream()
    if side is not None and _DEFER:
        K.defer_reduces_begin(side, grads)
    if _LN_DEFER and enabled():
        main = _current(grads.device.index)
        K.ln_defer_begin(main)
        _LN_STREAM[:] = [main]


def defer_flush():
    """before anything reads weight gradients the side stream produced (norm chunks, DP buckets, the join) -- called
    on the main stream, so the LayerNorm reduces flushed here are ordered before the reader's fork event"""
    if _LN_STREAM:
        from .. import kernels as K
        K.ln_defer_flush(_LN_STREAM[0])
    side = side_stream()
    if side is not None and _DEFER:
        from .. import kernels as K
        K.defer_reduces_flush(side)


def defer_end():
    side = side_stream()
    if _LN_STREAM:
        from .. import kernels as K
        main = _LN_STREAM.pop()
        if side is not None:
            # the last LayerNorm reduces go out on the side stream after everything queued on the main stream, so a
            # captured step (trainer/step_graph.py) still ends in one sink: the side chain's last node, which the
            # join hands back to the main stream
            side.wait_stream(main)
            K.ln_defer_end(main, launch=side)
        else:
            K.ln_defer_end(main)
    if side is not None and _DEFER:
        from .. import kernels as K
        K.defer_reduces_end(side)


def join():
    """make the current stream wait for all weight-gradient work queued so far."""
    side = side_stream()
    if side is not None:
        torch.cuda.current_stream().wait_stream(side)
    for h in _HAZARD:
        h.joined()


def after_side(fn):
    """run fn (e.g. an async all-reduce launch) ordered after both streams' work so far."""
    side = side_stream()
    if side is None:
        return fn()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        return fn()
