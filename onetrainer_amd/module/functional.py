"""torch.autograd.Functions over the HIP kernels (onetrainer_amd/kernels.py).

PyTorch hosts the tensors and the autograd graph; every forward/backward here launches the
hand-written gfx950 kernels.  Parameter gradients never go through autograd: each Function
receives a `PRef` (weight view + grad view in the FlatParamStore), writes the weight gradient
in place (overwrite, or accumulate inside a gradient-accumulation window) and calls
`store.mark_ready` so the DP reducer can launch that bucket's all-reduce while backward
continues.  The nn.Parameters are still passed as inputs so autograd connects the graph; their
returned gradient is None.
"""
from __future__ import annotations

import os

import torch

from .. import kernels as K
from . import streams as S


class PRef:
    """A (possibly fused) trainable tensor: value view, grad view, member names, store.
    Reading `w` orders the current stream after any optimizer chunk still updating it
    (FlatParamStore.wait_params: the update of step t overlaps step t+1's forward)."""
    __slots__ = ("store", "names", "_w", "g", "params", "_end")

    def __init__(self, store, names, shape=None):
        if isinstance(names, str):
            names = [names]
        self.store = store
        self.names = list(names)
        self._w = store.view(self.names, shape)
        self.g = store.view(self.names, shape, grad=True)
        self.params = tuple(store.params[n] for n in self.names)
        last = store.slots[self.names[-1]]
        self._end = last.offset + last.numel

    @property
    def w(self):
        if self.store.update_events is not None:
            self.store.wait_params(self._end)
        return self._w

    @property
    def trainable(self) -> bool:
        return self.store.trainable

    def acc(self) -> bool:
        return self.store.accumulate_into(self.names)

    def done(self):
        self.store.mark_ready(self.names)

    def write_f32(self, src_f32: torch.Tensor):
        """grad <- src (fp32 reduction result of a bias / norm-affine gradient)."""
        K.cast_f32_bf16(src_f32.reshape(-1).contiguous(), out=self.g.view(-1), accumulate=self.acc())
        self.done()


def _params(*refs):
    out = []
    for r in refs:
        if r is not None:
            out.extend(r.params)
    return out


def _rows(t: torch.Tensor) -> torch.Tensor:
    """2-D [rows, C] view of a token-major / NHWC tensor (keeps the row stride)."""
    if t.dim() == 2:
        return t
    return t.reshape(-1, t.shape[-1]) if t.is_contiguous() else t.view(-1, t.shape[-1])


def _kernel_rows(t: torch.Tensor) -> bool:
    """True when the kernels can read t in place as [rows, C] rows: unit channel stride, 16-byte aligned rows whose
    leading dims collapse onto one row stride (e.g. a channel slice of the up path's concat gradient)."""
    if t.stride(-1) != 1 or t.data_ptr() % 16 or t.dim() < 2 or t.stride(-2) % 8:
        return False
    exp = t.stride(-2)
    for d in range(t.dim() - 2, -1, -1):
        if t.shape[d] > 1 and t.stride(d) != exp:
            return False
        exp *= t.shape[d]
    return True


# ----------------------------------------------------------------------------------------------
class LinearFn(torch.autograd.Function):
    """y = x @ W^T (+b) (+residual) over the last dim; x any [..., K] with unit inner stride."""

    @staticmethod
    def forward(ctx, x, wref, bref, residual, *params):
        shp = x.shape
        x2 = _rows(x)
        r2 = _rows(residual) if residual is not None else None
        y = K.linear(x2, wref.w, bias=bref.w if bref is not None else None, residual=r2)
        ctx.save_for_backward(x2)
        ctx.wref, ctx.bref, ctx.has_res, ctx.xshape = wref, bref, residual is not None, shp
        return y.view(*shp[:-1], wref.w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        (x2,) = ctx.saved_tensors
        wref, bref = ctx.wref, ctx.bref
        dy2 = _rows(dy)
        if dy2.stride(1) != 1 or dy2.stride(0) % 8:
            dy2 = dy2.contiguous()
        btr = bref is not None and bref.trainable
        if wref.trainable or btr:
            with S.wgrad_region((dy2, x2)):       # weight gradients overlap the dgrad chain
                if wref.trainable:   # the bias gradient (sum of dy over tokens) rides in the same GEMM
                    K.linear_wgrad(dy2, x2, out=wref.g, accumulate=wref.acc(),
                                   bias_grad=bref.g.view(-1) if btr else None, bias_acc=btr and bref.acc())
                elif btr:
                    K.colsum(dy2, out=bref.g.view(1, -1), accumulate=bref.acc())
        dx = None
        if ctx.needs_input_grad[0]:
            dx = K.linear_dgrad(dy2, wref.w).view(ctx.xshape)
        if wref.trainable:
            wref.done()
        if btr:
            bref.done()
        dres = dy if ctx.has_res else None
        return (dx, None, None, dres) + (None,) * (len(ctx.needs_input_grad) - 4)


class PrecomputedLinearFn(torch.autograd.Function):
    """y = x W^T whose forward was computed already (one batched GEMM with its sibling layers, see
    UNet2DConditionModel._kv_batched); holder = [y].  Backward is LinearFn's (no bias / residual):
    weight gradient on the side stream, dx only when x needs it."""

    @staticmethod
    def forward(ctx, x, wref, holder, *params):
        x2 = _rows(x)
        ctx.save_for_backward(x2)
        ctx.wref, ctx.xshape = wref, x.shape
        y = holder[0]
        return y.view(*x.shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        (x2,) = ctx.saved_tensors
        wref = ctx.wref
        dy2 = _rows(dy)
        if dy2.stride(1) != 1 or dy2.stride(0) % 8:
            dy2 = dy2.contiguous()
        if wref.trainable:
            with S.wgrad_region((dy2, x2)):
                K.linear_wgrad(dy2, x2, out=wref.g, accumulate=wref.acc())
        dx = K.linear_dgrad(dy2, wref.w).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        if wref.trainable:
            wref.done()
        return (dx, None, None) + (None,) * (len(ctx.needs_input_grad) - 3)


def precomputed_linear(x, wref, y):
    return PrecomputedLinearFn.apply(x, wref, [y], *_params(wref))


# a LoRA linear whose input needs no gradient runs its whole backward on the weight-gradient stream
# (OTAMD_WGRAD_ONLY_SIDE=0: u = dy (sB) on the current stream, the A/B reference)
_WONLY_SIDE = os.environ.get("OTAMD_WGRAD_ONLY_SIDE", "1") != "0"


def linear(x, wref, bref=None, residual=None, lora=None):
    if lora is not None:
        return LoraLinearFn.apply(x, wref, bref, residual, lora, *lora.params, *_trainable_params(wref, bref))
    return LinearFn.apply(x, wref, bref, residual, *_params(wref, bref))


def _trainable_params(*refs):
    return [p for r in refs if r is not None and r.trainable for p in r.params]


class LoraLinearFn(torch.autograd.Function):
    """y = x W^T (+b) (+residual) + s * (x A^T) B^T with a frozen base (LoRAModule.forward,
    modules/module/LoRAModule.py:318-322).  Forward: one launch with t = x A^T accumulated in the base GEMM's K loop
    and [t | s B] as its second K segment (kernels.linear_lora; two launches where the plan does not allow it).
    Backward: u = dy (sB); dx = [dy | u] [W ; A] (one GEMM; at r = 32 on single-module and q|k|v sites u is
    accumulated inside it, kernels.linear_dgrad_lora); dA = u^T x; dB_p = s dy_p^T t_p per fused part; all adapter grads fp32."""

    @staticmethod
    def forward(ctx, x, wref, bref, residual, site, *params):
        shp = x.shape
        x2 = _rows(x)
        r2 = _rows(residual) if residual is not None else None
        t = torch.empty((x2.shape[0], site.down.shape[0]), dtype=x2.dtype, device=x2.device)
        y = K.linear_lora(x2, wref.w, bref.w if bref is not None else None, r2, site.down, site.up2, t, site.rank,
                          site.part_width)
        ctx.save_for_backward(x2, t)
        ctx.wref, ctx.bref, ctx.site, ctx.has_res, ctx.xshape = wref, bref, site, residual is not None, shp
        return y.view(*shp[:-1], wref.w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, t = ctx.saved_tensors
        wref, bref, site = ctx.wref, ctx.bref, ctx.site
        btr = bref is not None and bref.trainable
        need_dx = ctx.needs_input_grad[0]

        def wgrads(dy2, u):
            acc = site.acc()
            K.linear_wgrad(u, x2, out=site.g_down, accumulate=acc)
            r = site.rank
            for p, (g, (n0, n1)) in enumerate(zip(site.g_up, site.ranges)):
                K.linear_wgrad(dy2[:, n0:n1], t[:, p * r:(p + 1) * r], out=g, accumulate=acc, alpha=site.scale)
            if wref.trainable:
                K.linear_wgrad(dy2, x2, out=wref.g, accumulate=wref.acc())
            if btr:
                K.colsum(dy2, out=bref.g.view(1, -1), accumulate=bref.acc())

        dx = None
        if not need_dx and _WONLY_SIDE and S.side_stream() is not None:
            # no input gradient (the cross-attention K / V projection of text states that need none): u = dy (sB) is
            # only a weight-gradient operand, so the whole backward goes to the weight-gradient stream
            with S.wgrad_region((dy, x2, t)):
                dy2 = _rows(dy)
                if dy2.stride(1) != 1 or dy2.stride(0) % 8:
                    dy2 = dy2.contiguous()
                wgrads(dy2, K.linear_dgrad(dy2, site.up2))
        else:
            dy2 = _rows(dy)
            if dy2.stride(1) != 1 or dy2.stride(0) % 8:
                dy2 = dy2.contiguous()
            if need_dx and site.upT is not None:
                # one launch: u = dy (sB) inside the input-gradient GEMM's K loop (kernels.linear_dgrad_lora)
                u = torch.empty((dy2.shape[0], site.up2.shape[1]), dtype=dy2.dtype, device=dy2.device)
                dx = K.linear_dgrad_lora(dy2, wref.w, site.up2, site.down, site.upT, site.downT, u).view(ctx.xshape)
                with S.wgrad_region((dy2, x2, t, u)):
                    wgrads(dy2, u)
            else:
                u = K.linear_dgrad(dy2, site.up2)
                with S.wgrad_region((dy2, x2, t, u)):
                    wgrads(dy2, u)
                if need_dx:
                    dx = K.linear_dgrad(dy2, wref.w, lora=(u, site.down)).view(ctx.xshape)
        site.done()
        if wref.trainable:
            wref.done()
        if btr:
            bref.done()
        dres = dy if ctx.has_res else None
        return (dx, None, None, dres, None) + (None,) * (len(ctx.needs_input_grad) - 5)


class ConvFn(torch.autograd.Function):
    """NHWC conv 3x3 (pad 1), stride 1/2, optional virtual nearest-2x upsample of the input,
    epilogue + bias + rowvec[n] (ResnetBlock2D time-embedding projection) + residual."""

    @staticmethod
    def forward(ctx, x, wref, bref, rowvec, residual, stride, upsample, *params):
        y = K.conv2d(x, wref.w, bias=bref.w if bref is not None else None, stride=stride, pad=1, upsample=upsample,
                     residual=residual, rowvec=rowvec)
        ctx.save_for_backward(x)
        ctx.wref, ctx.bref, ctx.stride, ctx.upsample = wref, bref, stride, upsample
        ctx.has_rowvec, ctx.has_res = rowvec is not None, residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        wref, bref = ctx.wref, ctx.bref
        if dy.stride(3) != 1 or dy.stride(2) % 8 or dy.stride(1) != dy.stride(2) * dy.shape[2] \
                or dy.stride(0) != dy.stride(1) * dy.shape[1]:
            dy = dy.contiguous()
        N, H, W, _ = x.shape
        btr = bref is not None and bref.trainable
        if wref.trainable or btr:
            with S.wgrad_region((dy, x)):
                if wref.trainable:   # + the bias gradient from the same GEMM's dy images
                    K.conv2d_wgrad(dy, x, 3, ctx.stride, 1, upsample=ctx.upsample, out=wref.g, accumulate=wref.acc(),
                                   bias_grad=bref.g.view(-1) if btr else None, bias_acc=btr and bref.acc())
                elif btr:
                    K.colsum(dy, out=bref.g.view(1, -1), accumulate=bref.acc())
        dx = None
        if ctx.needs_input_grad[0]:
            if ctx.upsample:
                dup = K.conv2d_dgrad(dy, wref.w, (2 * H, 2 * W), 1, 1)
                dx = K.upsample2x_bwd(dup)
            else:
                dx = K.conv2d_dgrad(dy, wref.w, (H, W), ctx.stride, 1)
        drow = None
        P, Q = dy.shape[1], dy.shape[2]
        if ctx.has_rowvec:
            drow = K.colsum(dy, rows_per_group=P * Q, out=torch.empty((dy.shape[0], dy.shape[3]), dtype=torch.bfloat16,
                                                                       device=dy.device))
        if wref.trainable:
            wref.done()
        if btr:
            bref.done()
        dres = dy if ctx.has_res else None
        return (dx, None, None, drow, dres, None, None) + (None,) * (len(ctx.needs_input_grad) - 7)


class LoraConvFn(torch.autograd.Function):
    """ConvFn + LoRA (LoRAModule.py:142-155 conv branch): down = the base 3x3 geometry in->r,
    up = 1x1 r->out fused into the base conv GEMM as its second K segment; frozen base."""

    @staticmethod
    def forward(ctx, x, wref, bref, rowvec, residual, stride, upsample, site, *params):
        Ho, Wo = K.conv_out_hw(x.shape[1], x.shape[2], site.k, stride, 1, upsample)
        t = torch.empty((x.shape[0], Ho, Wo, site.down.shape[0]), dtype=x.dtype, device=x.device)
        y = K.conv2d_lora(x, wref.w, bref.w if bref is not None else None, stride, 1, upsample, residual, rowvec,
                          site.down, site.up2, t, site.rank)
        ctx.save_for_backward(x, t)
        ctx.wref, ctx.bref, ctx.stride, ctx.upsample, ctx.site = wref, bref, stride, upsample, site
        ctx.has_rowvec, ctx.has_res = rowvec is not None, residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, t = ctx.saved_tensors
        wref, bref, site = ctx.wref, ctx.bref, ctx.site
        if dy.stride(3) != 1 or dy.stride(2) % 8 or dy.stride(1) != dy.stride(2) * dy.shape[2] \
                or dy.stride(0) != dy.stride(1) * dy.shape[1]:
            dy = dy.contiguous()
        N, H, W, _ = x.shape
        _, P, Q, Cout = dy.shape
        M = N * P * Q
        dy2 = dy.reshape(M, Cout)
        r = site.rank
        u = K.linear_dgrad(dy2, site.up2).view(N, P, Q, r)          # dy (s B)
        btr = bref is not None and bref.trainable
        with S.wgrad_region((dy, x, t, u)):
            acc = site.acc()
            K.conv2d_wgrad(u, x, site.k, ctx.stride, 1, upsample=ctx.upsample, out=site.g_down, accumulate=acc)
            K.linear_wgrad(dy2, t.reshape(M, r), out=site.g_up[0], accumulate=acc, alpha=site.scale)
            if wref.trainable:
                K.conv2d_wgrad(dy, x, 3, ctx.stride, 1, upsample=ctx.upsample, out=wref.g, accumulate=wref.acc())
            if btr:
                K.colsum(dy, out=bref.g.view(1, -1), accumulate=bref.acc())
        dx = None
        if ctx.needs_input_grad[0]:
            if ctx.upsample:
                dup = K.conv2d_dgrad(dy, wref.w, (2 * H, 2 * W), 1, 1)
                K.conv2d_dgrad(u, site.down, (2 * H, 2 * W), 1, 1, out=dup, accumulate=True)
                dx = K.upsample2x_bwd(dup)
            else:
                dx = K.conv2d_dgrad(dy, wref.w, (H, W), ctx.stride, 1)
                K.conv2d_dgrad(u, site.down, (H, W), ctx.stride, 1, out=dx, accumulate=True)
        site.done()
        drow = None
        if ctx.has_rowvec:
            drow = K.colsum(dy, rows_per_group=P * Q, out=torch.empty((N, Cout), dtype=torch.bfloat16, device=dy.device))
        if wref.trainable:
            wref.done()
        if btr:
            bref.done()
        dres = dy if ctx.has_res else None
        return (dx, None, None, drow, dres, None, None, None) + (None,) * (len(ctx.needs_input_grad) - 8)


def conv(x, wref, bref=None, rowvec=None, residual=None, stride=1, upsample=False, lora=None):
    if lora is not None:
        return LoraConvFn.apply(x, wref, bref, rowvec, residual, stride, upsample, lora, *lora.params,
                                *_trainable_params(wref, bref))
    return ConvFn.apply(x, wref, bref, rowvec, residual, stride, upsample, *_params(wref, bref))


class GroupNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gref, bref, groups, eps, silu, *params):
        y, stats = K.groupnorm_fwd(x, gref.w, bref.w, groups, eps, silu)
        ctx.save_for_backward(x, *stats)
        ctx.gref, ctx.bref, ctx.groups, ctx.silu = gref, bref, groups, silu
        return y

    @staticmethod
    def backward(ctx, dy):
        x, *stats = ctx.saved_tensors
        tr = ctx.gref.trainable
        dx, _, _ = K.groupnorm_bwd(x, dy, ctx.gref.w, ctx.groups, ctx.silu, stats, dgamma=ctx.gref.g if tr else None,
                                   dbeta=ctx.bref.g if tr else None, param_acc=tr and ctx.gref.acc(),
                                   need_param_grads=tr)
        if tr:
            ctx.gref.done()
            ctx.bref.done()
        return (dx if ctx.needs_input_grad[0] else None,) + (None,) * (len(ctx.needs_input_grad) - 1)


def group_norm(x, gref, bref, groups, eps, silu):
    return GroupNormFn.apply(x, gref, bref, groups, eps, silu, *_params(gref, bref))


class GroupNormResFn(torch.autograd.Function):
    """(GroupNorm(+SiLU)(x), x) for a GroupNorm whose input also feeds a residual / shortcut (diffusers
    ResnetBlock2D: norm1 and the identity or conv_shortcut path; Transformer2DModel: norm and the proj_out
    residual).  The second output aliases x; backward receives both gradient contributions and sums them in
    the GroupNorm-backward apply pass (otamd_groupnorm_bwd_res) instead of leaving an autograd add kernel."""

    @staticmethod
    def forward(ctx, x, gref, bref, groups, eps, silu, *params):
        y, stats = K.groupnorm_fwd(x, gref.w, bref.w, groups, eps, silu)
        ctx.save_for_backward(x, *stats)
        ctx.gref, ctx.bref, ctx.groups, ctx.silu = gref, bref, groups, silu
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dres):
        x, *stats = ctx.saved_tensors
        tr = ctx.gref.trainable
        if dres is not None and not _kernel_rows(dres):   # strided rows (a concat-gradient slice) are read in place
            dres = dres.contiguous()
        if dy is None:   # only the residual use reached backward
            dy = torch.zeros_like(x)
        dx, _, _ = K.groupnorm_bwd(x, dy, ctx.gref.w, ctx.groups, ctx.silu, stats,
                                   dgamma=ctx.gref.g if tr else None, dbeta=ctx.bref.g if tr else None,
                                   param_acc=tr and ctx.gref.acc(), need_param_grads=tr, dres=dres)
        if tr:
            ctx.gref.done()
            ctx.bref.done()
        return (dx if ctx.needs_input_grad[0] else None,) + (None,) * (len(ctx.needs_input_grad) - 1)


def group_norm_res(x, gref, bref, groups, eps, silu):
    """-> (GroupNorm(+SiLU)(x), residual alias of x); see GroupNormResFn."""
    return GroupNormResFn.apply(x, gref, bref, groups, eps, silu, *_params(gref, bref))


class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gref, bref, eps, *params):
        y, stats = K.layernorm_fwd(x, gref.w, bref.w, eps)
        ctx.save_for_backward(x, *stats)
        ctx.gref, ctx.bref = gref, bref
        return y

    @staticmethod
    def backward(ctx, dy):
        x, *stats = ctx.saved_tensors
        if dy.stride(-1) != 1:
            dy = dy.contiguous()
        tr = ctx.gref.trainable
        if tr:   # dgamma / dbeta only feed the optimizer: side stream, like the GEMM weight gradients
            with S.wgrad_region((x, dy, *stats)):
                K.layernorm_param_grad(x, dy, stats, ctx.gref.g, ctx.bref.g, param_acc=ctx.gref.acc())
        dx, _, _ = K.layernorm_bwd(x, dy, ctx.gref.w, stats, need_param_grads=False)
        if tr:
            ctx.gref.done()
            ctx.bref.done()
        return (dx,) + (None,) * (len(ctx.needs_input_grad) - 1)


def layer_norm(x, gref, bref, eps=1e-5):
    return LayerNormFn.apply(x, gref, bref, eps, *_params(gref, bref))


class LayerNormResFn(torch.autograd.Function):
    """(LayerNorm(x), x) for a LayerNorm whose input is also the block's residual (diffusers
    BasicTransformerBlock: norm1/2/3 input = the residual of attn1/attn2 to_out and ff.net.2).  The
    second output aliases x; backward receives both gradient contributions and sums them inside the
    LayerNorm-backward pass (otamd_layernorm_bwd_res) instead of leaving an autograd add."""

    @staticmethod
    def forward(ctx, x, gref, bref, eps, *params):
        y, stats = K.layernorm_fwd(x, gref.w, bref.w, eps)
        ctx.save_for_backward(x, *stats)
        ctx.gref, ctx.bref = gref, bref
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dres):
        x, *stats = ctx.saved_tensors
        if dy.stride(-1) != 1:
            dy = dy.contiguous()
        tr = ctx.gref.trainable
        if dres is None:
            dx, _, _ = K.layernorm_bwd(x, dy, ctx.gref.w, stats, need_param_grads=False)
        else:
            if dres.stride(-1) != 1 or not dres.is_contiguous():
                dres = dres.contiguous()
            dx = K.layernorm_bwd_res(x, dy, dres, ctx.gref.w, stats)
        if tr:
            # dgamma / dbeta right after dx on this stream, while x and dy are still in the Infinity Cache: on
            # the weight-gradient stream they re-read HBM and slowed the critical-path dx pass by co-running
            # (SDXL 142.9 -> 141.4 ms/step, same-box A/B over two repetitions)
            K.layernorm_param_grad(x, dy, stats, ctx.gref.g, ctx.bref.g, param_acc=ctx.gref.acc())
            ctx.gref.done()
            ctx.bref.done()
        return (dx,) + (None,) * (len(ctx.needs_input_grad) - 1)


def layer_norm_res(x, gref, bref, eps=1e-5):
    """-> (LayerNorm(x), residual alias of x); see LayerNormResFn."""
    return LayerNormResFn.apply(x, gref, bref, eps, *_params(gref, bref))


class SelfAttnFn(torch.autograd.Function):
    """qkv [B, N, 3C] (fused projection output) -> o [B, N, C]."""

    @staticmethod
    def forward(ctx, qkv, heads):
        C = qkv.shape[-1] // 3
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        o, lse = K.attn_fwd(q, k, v, heads)
        ctx.save_for_backward(qkv, o, lse)
        ctx.heads = heads
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        do = do.contiguous()
        C = qkv.shape[-1] // 3
        dqkv = torch.empty_like(qkv)
        K.attn_bwd(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], o, lse, do, ctx.heads,
                   dq=dqkv[..., :C], dk=dqkv[..., C:2 * C], dv=dqkv[..., 2 * C:])
        return dqkv, None


# the cross-attention dK / dV chunk sum on the weight-gradient stream when only weight gradients consume dkv
# (OTAMD_CROSS_CAST_SIDE=0: on the current stream, the A/B reference)
_CROSS_CAST_SIDE = os.environ.get("OTAMD_CROSS_CAST_SIDE", "1") != "0"


class CrossAttnFn(torch.autograd.Function):
    """q [B, N, C], kv [B, L, 2C] -> o [B, N, C].  kv_wgrad_only: every consumer of dkv runs on the weight-gradient
    stream (kv from PrecomputedLinearFn, or from a LoRA projection, over text states that need no gradient), so the
    one-pass backward's dK / dV chunk sum (attn_dkv_cast) is queued there too, off the critical stream."""

    @staticmethod
    def forward(ctx, q, kv, heads, kv_wgrad_only=False):
        C = q.shape[-1]
        o, lse = K.attn_fwd(q, kv[..., :C], kv[..., C:], heads)
        ctx.save_for_backward(q, kv, o, lse)
        ctx.heads = heads
        ctx.kv_wgrad_only = kv_wgrad_only
        return o

    @staticmethod
    def backward(ctx, do):
        q, kv, o, lse = ctx.saved_tensors
        do = do.contiguous()
        C = q.shape[-1]
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        # the side stream only when every reader of dkv is queued there: PrecomputedLinearFn's weight gradient reads
        # dkv in place (rows of 2C elements, 16-byte aligned when C % 4 == 0; otherwise its main-stream
        # .contiguous() copy would read dkv before the cast) and kv_wgrad_only says no dx (text states need none)
        side = S.side_stream() if (ctx.kv_wgrad_only and _CROSS_CAST_SIDE and ctx.needs_input_grad[1]
                                   and C % 4 == 0) else None
        K.attn_bwd(q, kv[..., :C], kv[..., C:], o, lse, do, ctx.heads, dq=dq, dk=dkv[..., :C], dv=dkv[..., C:],
                   cast_stream=side)
        if side is not None:
            dkv.record_stream(side)
            S.note_side((dkv,))
        return dq, (dkv if ctx.needs_input_grad[1] else None), None, None


class GEGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h):
        ctx.save_for_backward(h)
        return K.geglu_fwd(h)

    @staticmethod
    def backward(ctx, dy):
        (h,) = ctx.saved_tensors
        return K.geglu_bwd(h, dy.contiguous())


class SiLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return K.silu_fwd(x.contiguous())

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return K.silu_bwd(x.contiguous(), dy.contiguous())


class ConcatFn(torch.autograd.Function):
    """channel concat of two NHWC tensors (UNet up-block skip connection)."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.ca = a.shape[-1]
        return K.concat_channels(a, b)

    @staticmethod
    def backward(ctx, dy):
        return dy[..., :ctx.ca], dy[..., ctx.ca:]


class MSELossFn(torch.autograd.Function):
    """ModelSetupDiffusionLossMixin.__unmasked_losses + _diffusion_losses + .mean() (+ /GA)."""

    @staticmethod
    def forward(ctx, pred, target, loss_weight, timestep, coeffs, loss_fn, gamma, v_pred, ga, mse_strength, scale,
                grad_scale=1.0, num_t=1000):
        loss, coef, losses = K.mse_loss(pred, target, loss_weight, mse_strength=mse_strength, scale=scale,
                                        loss_fn=loss_fn, gamma=gamma, v_pred=v_pred, ga=ga, timestep=timestep,
                                        coeffs=coeffs, num_t=num_t)
        ctx.save_for_backward(pred, target, coef)
        ctx.losses = losses
        ctx.grad_scale = grad_scale
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        pred, target, coef = ctx.saved_tensors
        gd = g.reshape(1).float()
        if ctx.grad_scale != 1.0:   # data-parallel: fold 1/world into the loss gradient (sum all-reduce = mean)
            gd = gd * ctx.grad_scale
        return (K.mse_grad(pred, target, coef, grad_out=gd.contiguous()),) + (None,) * 12
