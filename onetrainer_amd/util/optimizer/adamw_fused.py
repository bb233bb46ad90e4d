"""Fused multi-tensor AdamW (+ bf16 stochastic rounding) over a FlatParamStore.

Drop-in for what the reference builds at modules/util/create.py:509-534:
    torch.optim.AdamW(params, lr, betas, weight_decay, eps, foreach=False, fused=False)
    patch_adamw(optimizer, stochastic_rounding)          # modules/util/optimizer/adamw_extensions.py:202-205
plus the global clip the trainer applies before step() (modules/trainer/GenericTrainer.py:712-713).
Same optimizer contract: param_groups with 'lr' (LambdaLR drives it), step(),
zero_grad(set_to_none), state_dict()/load_state_dict() (torch AdamW layout: per-param 'step',
'exp_avg', 'exp_avg_sq'), step_parameter(p, group, i).  The arithmetic is one launch over the
flat store (csrc/adamw.hip) instead of ~8 torch ops per tensor.

Overlap (opt-in, OTAMD_OPT_OVERLAP=1; bf16 stores of >= 64 M elements): step() runs the update on
its own stream in 16 parameter-range chunks (layout = forward order) and records an event per chunk
in the store; the next forward's kernels wait only for the chunk holding their weights
(FlatParamStore.wait_params via PRef.w), so the 36 GB optimizer pass (SDXL: ~6 ms of HBM time)
runs beside the compute-bound forward GEMMs instead of in front of them.  Chunked launches give the
bits of one whole-store launch (global element indices for groups and stochastic rounding).
Readers of the parameters outside the train step call store.wait_params() (state_dict, savers and
backups do).  Measured on the SDXL step (MI355X): no gain (151.1 vs 150.6 ms p50) -- a 256x256 GEMM
workgroup takes a whole CU's register file, so the update only time-slices CUs with the forward.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import torch

from ... import _lib
from ... import kernels as K


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, store, param_groups, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 stochastic_rounding=True, seed=0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=False, capturable=False, differentiable=False, fused=False)
        super().__init__(param_groups, defaults)
        self.store = store
        self.stochastic_rounding = stochastic_rounding
        self.seed = seed
        # fp32 master weights (module/param_store.py `master`): fp32 moments, the reference's fp32 AdamW path
        # (adamw_extensions.py:125-148 without stochastic rounding, which applies to bf16 parameters only)
        self.master = getattr(store, "master", None)
        self.exp_avg = torch.zeros_like(self.master if self.master is not None else store.data)
        self.exp_avg_sq = torch.zeros_like(self.exp_avg)
        self._norm_dtype = K.grad_norm_dtype(store.grad, self.master is not None) if store.grad is not None else 0
        self._ptr2name = {store.params[n].data_ptr(): n for n in store.order}
        self._ranges = []
        for g in self.param_groups:
            offs = []
            for p in g["params"]:
                s = store.slots[self._ptr2name[p.data_ptr()]]
                offs.append((s.offset, s.offset + s.numel))
            b, e = min(o[0] for o in offs), max(o[1] for o in offs)
            covered = sum(o[1] - o[0] for o in offs)
            span = [s for s in store.order if b <= store.slots[s].offset < e]
            if len(span) != len(offs):
                raise ValueError("each optimizer param group must be a contiguous range of the flat store")
            self._ranges.append((b, e))
            del covered
        self.steps = [0 for _ in self.param_groups]
        # per-tensor chunk table for the global grad norm
        chunks = []
        for ti, n in enumerate(store.order):
            s = store.slots[n]
            for c0 in range(s.offset, s.offset + s.numel, 1 << 16):
                chunks.append((c0, min(s.offset + s.numel, c0 + (1 << 16)), ti))
        arr = (_lib.NormChunk * len(chunks))()
        for i, (b, e, t) in enumerate(chunks):
            arr[i].begin, arr[i].end, arr[i].tensor = b, e, t
        raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        self._chunks = raw.to(store.device)
        self._n_chunks = len(chunks)
        self._tensor_sq = torch.zeros(len(store.order), dtype=torch.float64, device=store.device)
        self._chunk_sq = torch.zeros(max(1, len(chunks)), dtype=torch.float64, device=store.device)   # one slot per chunk
        self.clip_out = torch.zeros(2, dtype=torch.float32, device=store.device)   # [coef, total norm]
        self._chunk_tensor = [c[2] for c in chunks]
        self.norm_overlap = None   # OverlappedGradNorm, attached by the trainer (single process, clip on)
        # overlapped update: chunk boundaries on tensor boundaries, ~numel / 16 each
        self.overlap = (store.device.type == "cuda" and store.dtype == torch.bfloat16 and store.numel >= (1 << 26)
                        and self.master is None and os.environ.get("OTAMD_OPT_OVERLAP", "0") == "1")
        self._opt_chunks = []
        if self.overlap:
            # chunk ends at 1/256, 1/128, ..., 1/16 of the store, then every 1/16 (tensor boundaries): the forward's first
            # layers wait only for a small first chunk, the rest of the update runs beside them
            ends = [store.numel >> k for k in range(8, 4, -1)] + [store.numel * i // 16 for i in range(1, 17)]
            b, t = 0, 0
            for n in store.order:
                s = store.slots[n]
                e = (s.offset + s.numel + 7) // 8 * 8
                if t < len(ends) and e >= ends[t]:
                    self._opt_chunks.append((b, e))
                    b = e
                    while t < len(ends) and ends[t] <= e:
                        t += 1
            if b < store.numel:
                self._opt_chunks.append((b, store.numel))
            self._stream = torch.cuda.Stream(device=store.device)

    # --- clip_grad_norm_ (GenericTrainer.py:712-713) ----------------------------------------------
    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """computes the clip coefficient on device; it is applied inside the next step()."""
        self.store.wait_params()   # the previous (overlapped) update still reads grads / clip_out
        nt = len(self.store.order)
        if self.norm_overlap is not None and self.norm_overlap.take():   # sums accumulated during backward
            if _NORM_CHECK:   # debug: every overlapped chunk sum against the same pass over the final gradients
                ref = torch.empty_like(self._chunk_sq)
                _lib.check(_lib.lib().otamd_grad_sqnorm_chunks(self.store.grad.data_ptr(), self._norm_dtype,
                                                               self._chunks.data_ptr(), 0, self._n_chunks,
                                                               ref.data_ptr(), K.stream_handle()), "norm check")
                bad = (ref != self._chunk_sq[:self._n_chunks]).nonzero().flatten().tolist()
                if bad:
                    names = sorted({self.store.order[self._chunk_tensor[c]] for c in bad})
                    print(f"[norm check] {len(bad)} of {self._n_chunks} overlapped chunk sums differ from the final "
                          f"gradients': {names[:12]}", flush=True)
            _lib.check(_lib.lib().otamd_grad_clip_finalize(self._chunks.data_ptr(), self._n_chunks,
                                                           self._chunk_sq.data_ptr(), self._tensor_sq.data_ptr(), nt,
                                                           float(max_norm), self._norm_dtype,
                                                           self.clip_out.data_ptr(), K.stream_handle()),
                       "otamd_grad_clip_finalize")
        else:
            K.grad_clip_coef(self.store.grad, self._chunks, self._n_chunks, self._chunk_sq, self._tensor_sq, nt,
                             max_norm, self.clip_out, fp32_semantics=self.master is not None)
        self._pending_clip = True
        return self.clip_out[1]

    def _groups_struct(self, idx_list, steps=None):
        arr = []
        for k, gi in enumerate(idx_list):
            g = self.param_groups[gi]
            if steps is None:
                self.steps[gi] += 1
                step = self.steps[gi]
            else:
                step = steps[k]
            lr = float(g["lr"])
            beta1, beta2 = g["betas"]
            bc1 = 1 - beta1 ** step
            bc2 = 1 - beta2 ** step
            s = _lib.AdamwGroup()
            s.begin, s.end = self._ranges[gi]
            s.wd_factor = 1 - lr * g["weight_decay"]
            s.one_minus_beta1 = 1 - beta1
            s.beta2 = beta2
            s.one_minus_beta2 = 1 - beta2
            s.bc2_sqrt = math.sqrt(bc2)
            s.eps = g["eps"]
            s.neg_step_size = -(lr / bc1)
            arr.append(s)
        order = sorted(range(len(arr)), key=lambda i: arr[i].begin)
        return [arr[i] for i in order]

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        groups = self._groups_struct(range(len(self.param_groups)))
        clip = self.clip_out if getattr(self, "_pending_clip", False) else None
        self._pending_clip = False
        st = self.store
        if self.master is not None:
            K.adamw_master(self.master, st.grad, self.exp_avg, self.exp_avg_sq, st.data, groups, clip_coef=clip)
        elif st.dtype == torch.bfloat16:
            self.seed = (self.seed * 6364136223846793005 + 1442695040888963407) & 0xFFFFFFFFFFFFFFFF
            if self.overlap:
                st.wait_params()                                   # a previous update still in flight
                s = self._stream
                s.wait_stream(torch.cuda.current_stream())         # grads reduced, clip coefficient ready
                events = []
                with torch.cuda.stream(s):
                    for b, e in self._opt_chunks:
                        K.adamw_bf16(st.data, st.grad, self.exp_avg, self.exp_avg_sq, groups, clip_coef=clip,
                                     stochastic_rounding=self.stochastic_rounding, seed=self.seed, begin=b, end=e)
                        ev = torch.cuda.Event()
                        ev.record(s)
                        events.append((e, ev))
                st.set_update_events(events)
            else:
                K.adamw_bf16(st.data, st.grad, self.exp_avg, self.exp_avg_sq, groups, clip_coef=clip,
                             stochastic_rounding=self.stochastic_rounding, seed=self.seed)
        else:
            K.adamw_f32(st.data, st.grad, self.exp_avg, self.exp_avg_sq, groups, clip_coef=clip)
        return loss

    def step_parameter(self, p, group, i):
        """fused-back-pass API (adamw_extensions.py:202-205): update one parameter tensor."""
        self.store.wait_params()
        gi = self.param_groups.index(group)
        name = self._ptr2name[p.data_ptr()]
        s = self.store.slots[name]
        if not hasattr(self, "_pstep"):
            self._pstep = {}
        self._pstep[name] = self._pstep.get(name, self.steps[gi]) + 1
        saved = self._ranges[gi]
        self._ranges[gi] = (s.offset, s.offset + s.numel)
        try:
            groups = self._groups_struct([gi], steps=[self._pstep[name]])
        finally:
            self._ranges[gi] = saved
        st = self.store
        b, e = s.offset // 8 * 8, (s.offset + s.numel + 7) // 8 * 8   # this tensor only (the store pads to 8)
        if self.master is not None:
            K.adamw_master(self.master, st.grad, self.exp_avg, self.exp_avg_sq, st.data, groups, begin=b, end=e)
            return
        K.adamw_bf16(st.data, st.grad, self.exp_avg, self.exp_avg_sq, groups, clip_coef=None,
                     stochastic_rounding=self.stochastic_rounding, seed=self.seed, begin=b, end=e)

    def zero_grad(self, set_to_none: bool = True):
        """grads are views of the flat store that the next backward overwrites; nothing to clear."""
        self.store.accumulating = False

    # --- torch AdamW-compatible state -------------------------------------------------------------
    def state_dict(self):
        self.store.wait_params()
        state = {}
        idx = 0
        groups = []
        for gi, g in enumerate(self.param_groups):
            ids = []
            for p in g["params"]:
                s = self.store.slots[self._ptr2name[p.data_ptr()]]
                sl = slice(s.offset, s.offset + s.numel)
                state[idx] = {"step": torch.tensor(float(self.steps[gi])),
                              "exp_avg": self.exp_avg[sl].view(s.shape).clone(),
                              "exp_avg_sq": self.exp_avg_sq[sl].view(s.shape).clone()}
                ids.append(idx)
                idx += 1
            gd = {k: v for k, v in g.items() if k != "params"}
            gd["params"] = ids
            groups.append(gd)
        # the stochastic-rounding stream position, so that a resumed run rounds like an uninterrupted one
        return {"state": state, "param_groups": groups, "sr_seed": int(self.seed)}

    def load_state_dict(self, sd):
        self.store.wait_params()
        if "sr_seed" in sd:
            self.seed = int(sd["sr_seed"])
        idx = 0
        for gi, (g, gsd) in enumerate(zip(self.param_groups, sd["param_groups"])):
            for k, v in gsd.items():
                if k != "params":
                    g[k] = v
            for p, pid in zip(g["params"], gsd["params"]):
                s = self.store.slots[self._ptr2name[p.data_ptr()]]
                st = sd["state"].get(pid)
                if st:
                    sl = slice(s.offset, s.offset + s.numel)
                    self.exp_avg[sl].copy_(st["exp_avg"].reshape(-1))
                    self.exp_avg_sq[sl].copy_(st["exp_avg_sq"].reshape(-1))
                    self.steps[gi] = int(float(st["step"]))
                idx += 1


_NORM_CHECK = os.environ.get("OTAMD_NORM_CHECK") == "1"


class OverlappedGradNorm:
    """clip_grad_norm_'s squared-norm pass spread over the backward.  Single process: gradient ranges of about
    `bucket_bytes` (whole tensors, reverse layout order = the order backward finishes them) are summed on the
    weight-gradient stream as soon as every tensor in the range has its gradient -- the stream then waits for
    the dgrad chain's position, so both streams' writes are ordered before the read.  clip_grad_norm_ then only
    folds the per-chunk sums into per-tensor ones in chunk order (otamd_grad_clip_finalize) instead of reading
    the whole gradient buffer (SDXL: 5.1 GB, ~0.9 ms) after backward.  The sums are fp64, one slot per chunk
    (no atomics: the same bits every run), and the coefficient is formed with torch's bf16 roundings exactly as
    otamd_grad_clip_coef does.  Ranges with a tensor that received no gradient are
    summed after finish_backward has zeroed it.  Data parallel (`reducer`): the norm must see the all-reduced
    gradients, so the ranges are the reducer's buckets and each is summed on the reducer's post stream right after
    its collective completes (trainer/ddp.py reduced_hooks); only the last bucket's sums follow the backward.
    OTAMD_NORM_OVERLAP=0 disables it."""

    def __init__(self, opt: FusedAdamW, bucket_bytes: int = 64 << 20, reducer=None):
        self.opt = opt
        self.dp = reducer is not None
        store = opt.store
        limit = max(1, bucket_bytes // store.grad.element_size())
        t_chunks: dict = {}
        for ci, ti in enumerate(opt._chunk_tensor):
            b, e = t_chunks.get(ti, (ci, ci))
            t_chunks[ti] = (min(b, ci), max(e, ci + 1))
        self.buckets = []   # (first chunk, end chunk, names)
        if self.dp:
            t_index = {n: ti for ti, n in enumerate(store.order)}
            for _, _, names in reducer.buckets:
                spans = [t_chunks[t_index[n]] for n in names if t_index[n] in t_chunks]
                self.buckets.append((min(b for b, _ in spans) if spans else None,
                                     max(e for _, e in spans) if spans else None, list(names)))
            self.armed = False
            self.ready = False
            reducer.reduced_hooks.append(self._on_reduced)
            return
        cur, c_lo, c_hi, size = [], None, None, 0
        for ti in reversed(range(len(store.order))):
            name = store.order[ti]
            n = store.slots[name].numel
            if cur and size + n > limit:
                self.buckets.append((c_lo, c_hi, cur))
                cur, size = [], 0
            if not cur:
                c_lo, c_hi = None, None
            if ti in t_chunks:   # a tensor with no norm chunks (numel 0) must not stretch the bucket's range
                b, e = t_chunks[ti]
                c_lo = b if c_lo is None else min(c_lo, b)
                c_hi = e if c_hi is None else max(c_hi, e)
            cur.append(name)
            size += n
        if cur:
            self.buckets.append((c_lo, c_hi, cur))
        self.bucket_of = {n: bi for bi, (_, _, names) in enumerate(self.buckets) for n in names}
        self.armed = False
        self.ready = False
        self._ev = torch.cuda.Event()
        store.ready_hooks.append(self._on_ready)

    def arm(self, update_step: bool):
        """before the backward of a step: only the update step's gradients are final."""
        self.armed = update_step
        self.ready = False
        self.pending = [len(b[2]) for b in self.buckets]
        self._seen = set()
        self.launched = [False] * len(self.buckets)   # every bucket's chunk slots are rewritten each armed step

    def _launch(self, bi, side):
        self.launched[bi] = True
        c0, c1, _ = self.buckets[bi]
        if c0 is None:   # only empty tensors: nothing to sum
            return
        opt = self.opt
        g = opt.store.grad
        dtype = opt._norm_dtype
        if side is not None:
            from ...module import streams as S
            S.defer_flush()   # the bucket's deferred split-K reduces (module/streams.py) before its norms
            self._ev.record(torch.cuda.current_stream())
            side.wait_event(self._ev)
            with torch.cuda.stream(side):
                _lib.check(_lib.lib().otamd_grad_sqnorm_chunks(g.data_ptr(), dtype, opt._chunks.data_ptr(), c0, c1,
                                                               opt._chunk_sq.data_ptr(), K.stream_handle()),
                           "otamd_grad_sqnorm_chunks")
        else:
            _lib.check(_lib.lib().otamd_grad_sqnorm_chunks(g.data_ptr(), dtype, opt._chunks.data_ptr(), c0, c1,
                                                           opt._chunk_sq.data_ptr(), K.stream_handle()),
                       "otamd_grad_sqnorm_chunks")

    def _on_reduced(self, bi):
        """data parallel: bucket bi holds the global sum (on the reducer's post stream, the current stream here)."""
        if self.armed:
            self._launch(bi, None)

    def _on_ready(self, names):
        if not self.armed:
            return
        pending, bucket_of = self.pending, self.bucket_of
        if _NORM_CHECK:   # debug: a gradient marked twice, or after its range was summed, would race the norm pass
            for n in names:
                if n in self._seen:
                    raise RuntimeError(f"overlapped grad norm: {n} marked ready twice in one step")
                if self.launched[bucket_of[n]]:
                    raise RuntimeError(f"overlapped grad norm: {n} marked ready after its range was summed")
                self._seen.add(n)
        for n in names:
            bi = bucket_of[n]
            pending[bi] -= 1
            if pending[bi] == 0 and not self.launched[bi]:
                from ...module import streams as S
                self._launch(bi, S.side_stream())

    def finish(self):
        """after finish_backward (streams joined, grads of untouched tensors zeroed): sum what is left."""
        if not self.armed:
            return
        for bi in range(len(self.buckets)):
            if not self.launched[bi]:
                if self.dp:   # every reducer bucket goes out in reducer.finish(), which runs before this
                    raise RuntimeError("overlapped grad norm: bucket %d was not all-reduced this step" % bi)
                self._launch(bi, None)
        # every chunk slot is rewritten on an armed step: the finalize never sees an earlier step's sums
        assert all(self.launched), "overlapped grad norm: a bucket was not summed this step"
        self.ready = True

    def take(self) -> bool:
        """True once per armed step whose sums are complete (consumed by clip_grad_norm_)."""
        r = self.ready
        self.ready = False
        self.armed = False
        return r
