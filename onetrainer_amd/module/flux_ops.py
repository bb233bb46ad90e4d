"""autograd Functions of the FLUX.1 transformer over the HIP kernels (csrc/flux.hip, attention.hip,
the GEMM engine).  Activations are rows r = t * B + b of the joint sequence [text ; image]
(module/flux.py), so a stream is a row block [r0, r1) and the joint attention reads q / k / v
in place with token stride B * ld and batch stride ld.

Modulation.  All adaLN / gate vectors of the network come from one [B, NMOD] GEMM output
(`emb`).  Its consumers write their gradient chunks straight into a shared buffer (ModState.d,
each column range written by exactly one consumer kernel) and exactly one of them hands that
buffer to autograd as emb's gradient -- the engine runs the modulation GEMM's backward only after
every consumer has run, so no per-consumer full-size gradient is ever materialised or summed.
"""
from __future__ import annotations

import torch

from .. import kernels as K
from . import streams as S
from .functional import _trainable_params


class ModState:
    """shared gradient buffer of a modulation output (see module docstring)."""

    def __init__(self, emb: torch.Tensor):
        self.d = torch.empty_like(emb)
        self._owner = False
        self.side = False   # emb came from the weight-gradient stream (module/flux.py): the adaLN dmod sums go there

    def claim(self) -> bool:
        if self._owner:
            return False
        self._owner = True
        return True


def _seg_params(segs):
    out = []
    for s in segs:
        wref, bref, site = s[2], s[3], s[4]
        if site is not None:
            out.extend(site.params)
        out.extend(_trainable_params(wref, bref))
    return out


class RowsLinearFn(torch.autograd.Function):
    """y[r0:r1] = x[r0:r1] W_s^T + b_s (+ LoRA_s) for row segments s (the two streams of a double
    block); one joint output buffer, no concat."""

    @staticmethod
    def forward(ctx, x, segs, *params):
        R = x.shape[0]
        N = segs[0][2].w.shape[0]
        y = torch.empty((R, N), dtype=torch.bfloat16, device=x.device)
        ts = []
        for r0, r1, wref, bref, site in segs:
            xs = x[r0:r1]
            if site is not None:
                t = K.linear(xs, site.down)
                K.linear(xs, wref.w, bias=bref.w if bref is not None else None, lora=(t, site.up2), out=y[r0:r1])
                ts.append(t)
            else:
                K.linear(xs, wref.w, bias=bref.w if bref is not None else None, out=y[r0:r1])
                ts.append(None)
        ctx.save_for_backward(x)
        ctx.segs, ctx.ts = segs, ts
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        if dy.stride(1) != 1 or dy.stride(0) % 8:
            dy = dy.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        for (r0, r1, wref, bref, site), t in zip(ctx.segs, ctx.ts):
            dys, xs = dy[r0:r1], x[r0:r1]
            btr = bref is not None and bref.trainable
            u = K.linear_dgrad(dys, site.up2) if site is not None else None
            if site is not None or wref.trainable or btr:
                with S.wgrad_region((dys, xs, t, u)):
                    if site is not None:
                        acc = site.acc()
                        K.linear_wgrad(u, xs, out=site.g_down, accumulate=acc)
                        rk = site.rank
                        for p, (g, (n0, n1)) in enumerate(zip(site.g_up, site.ranges)):
                            K.linear_wgrad(dys[:, n0:n1], t[:, p * rk:(p + 1) * rk], out=g, accumulate=acc,
                                           alpha=site.scale)
                    if wref.trainable:   # bias gradient fused into the weight-gradient GEMM
                        K.linear_wgrad(dys, xs, out=wref.g, accumulate=wref.acc(),
                                       bias_grad=bref.g.view(-1) if btr else None, bias_acc=btr and bref.acc())
                    elif btr:
                        K.colsum(dys, out=bref.g.view(1, -1), accumulate=bref.acc())
            if dx is not None:
                if site is not None:
                    K.linear_dgrad(dys, wref.w, lora=(u, site.down), out=dx[r0:r1])
                else:
                    K.linear_dgrad(dys, wref.w, out=dx[r0:r1])
            if site is not None:
                site.done()
            if wref.trainable:
                wref.done()
            if btr:
                bref.done()
        return (dx, None) + (None,) * (len(ctx.needs_input_grad) - 2)


def rows_linear(x, segs):
    """segs: [(r0, r1, wref, bref, lora_site | None)]"""
    return RowsLinearFn.apply(x, segs, *_seg_params(segs))


def _dmod_side(ctx, x, dy, emb):
    """the adaLN's modulation-gradient sums on the weight-gradient stream, where the modulation GEMM's backward (its
    only reader) runs: they leave the dx chain"""
    with S.wgrad_region((x, dy) + tuple(t for st in ctx.stats for t in st)):
        for (r0, r1, sh, sc), st in zip(ctx.segs, ctx.stats):
            K.adaln_dmod(x[r0:r1], dy[r0:r1], emb, sh, sc, ctx.B, st, ctx.state.d)


class AdaLNFn(torch.autograd.Function):
    """y[r0:r1] = LN(x[r0:r1]) * (1 + emb[b, scale_off:]) + emb[b, shift_off:] per row segment."""

    @staticmethod
    def forward(ctx, x, emb, state, segs, B):
        y = torch.empty_like(x)
        stats = []
        for r0, r1, sh, sc in segs:
            _, st = K.adaln_fwd(x[r0:r1], emb, sh, sc, B, out=y[r0:r1])
            stats.append(st)
        ctx.save_for_backward(x, emb)
        ctx.stats, ctx.state, ctx.segs, ctx.B = stats, state, segs, B
        ctx.owner = state.claim()
        return y

    @staticmethod
    def backward(ctx, dy):
        x, emb = ctx.saved_tensors
        if dy.stride(1) != 1:
            dy = dy.contiguous()
        dx = torch.empty_like(x)
        side = ctx.state.side
        for (r0, r1, sh, sc), st in zip(ctx.segs, ctx.stats):
            K.adaln_bwd(x[r0:r1], dy[r0:r1], emb, sh, sc, ctx.B, st, dmod=None if side else ctx.state.d, dx=dx[r0:r1])
        if side:
            _dmod_side(ctx, x, dy, emb)
        return dx, (ctx.state.d if ctx.owner else None), None, None, None


class AdaLNResFn(torch.autograd.Function):
    """(AdaLN(x), residual alias of x) for an adaLN whose input is also the block's residual (the gated add after the
    attention / MLP branch): backward receives both gradient contributions and sums them inside the adaLN dx pass
    (otamd_adaln_bwd_res) instead of leaving autograd a separate add."""

    @staticmethod
    def forward(ctx, x, emb, state, segs, B):
        y = torch.empty_like(x)
        stats = []
        for r0, r1, sh, sc in segs:
            _, st = K.adaln_fwd(x[r0:r1], emb, sh, sc, B, out=y[r0:r1])
            stats.append(st)
        ctx.save_for_backward(x, emb)
        ctx.stats, ctx.state, ctx.segs, ctx.B = stats, state, segs, B
        ctx.owner = state.claim()
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dres):
        x, emb = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(x)
        if dy.stride(1) != 1:
            dy = dy.contiguous()
        if dres is not None and (dres.stride(1) != 1 or dres.stride(0) % 8):
            dres = dres.contiguous()
        dx = torch.empty_like(x)
        side = ctx.state.side
        for (r0, r1, sh, sc), st in zip(ctx.segs, ctx.stats):
            K.adaln_bwd(x[r0:r1], dy[r0:r1], emb, sh, sc, ctx.B, st, dmod=None if side else ctx.state.d, dx=dx[r0:r1],
                        dres=dres[r0:r1] if dres is not None else None)
        if side:
            _dmod_side(ctx, x, dy, emb)
        return dx, (ctx.state.d if ctx.owner else None), None, None, None


class GatedAddFn(torch.autograd.Function):
    """out[r0:r1] = x[r0:r1] + emb[b, gate_off:] * y[r0:r1] per row segment."""

    @staticmethod
    def forward(ctx, x, y, emb, state, segs, B):
        out = torch.empty_like(x)
        for r0, r1, g in segs:
            K.gated_add_fwd(x[r0:r1], y[r0:r1], emb, g, B, out=out[r0:r1])
        ctx.save_for_backward(y, emb)
        ctx.state, ctx.segs, ctx.B = state, segs, B
        ctx.owner = state.claim()
        return out

    @staticmethod
    def backward(ctx, dout):
        y, emb = ctx.saved_tensors
        if dout.stride(1) != 1:
            dout = dout.contiguous()
        dy = torch.empty_like(y)
        # (with the modulation branch on the weight-gradient stream the gate sums stay here, fused with dy: splitting
        # them off measured neutral, profiles/r6_flux_mod_side_ab.txt)
        for r0, r1, g in ctx.segs:
            K.gated_add_bwd(dout[r0:r1], y[r0:r1], emb, g, ctx.B, ctx.state.d, dy=dy[r0:r1])
        return dout, dy, (ctx.state.d if ctx.owner else None), None, None, None


def _tok_view(buf: torch.Tensor, col: int, D: int, B: int, T: int) -> torch.Tensor:
    """[B, T, D] attention view of columns [col, col + D) of rows r = t*B + b of a [T*B, ld] buffer."""
    ld = buf.stride(0)
    return buf.as_strided((B, T, D), (ld, B * ld, 1), buf.storage_offset() + col)


def _norm_w(refs):
    return tuple(r.w if r is not None else None for r in refs)


def _norm_g(refs):
    return tuple(r.g if (r is not None and r.trainable) else None for r in refs)


def _norm_done(refs, acc):
    for r in refs:
        if r is not None and r.trainable:
            r.done()


def _norm_acc(refs):
    return any(r is not None and r.trainable and r.acc() for r in refs)


class JointAttnFn(torch.autograd.Function):
    """double block: qkv [T*B, 3D] (text rows use the add_*_proj outputs) -> RMSNorm q/k (text rows:
    norm_added_*) + RoPE -> joint attention -> o [T*B, D]."""

    @staticmethod
    def forward(ctx, qkv, geo, norms, rope, *params):
        T, B, H, L = geo
        D = H * 128
        cs, sn = rope
        qk = K.qknorm_rope_fwd(qkv, 0, D, H, B, L, _norm_w(norms), cs, sn)
        o = torch.empty((T * B, D), dtype=torch.bfloat16, device=qkv.device)
        _, lse = K.attn_fwd(_tok_view(qk, 0, D, B, T), _tok_view(qk, D, D, B, T), _tok_view(qkv, 2 * D, D, B, T), H,
                            out=_tok_view(o, 0, D, B, T))
        ctx.save_for_backward(qkv, qk, o, lse)
        ctx.geo, ctx.norms, ctx.rope = geo, norms, rope
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, qk, o, lse = ctx.saved_tensors
        T, B, H, L = ctx.geo
        D = H * 128
        cs, sn = ctx.rope
        if do.stride(1) != 1 or do.stride(0) % 8:
            do = do.contiguous()
        dqk = torch.empty_like(qk)
        dqkv = torch.empty_like(qkv)
        K.attn_bwd(_tok_view(qk, 0, D, B, T), _tok_view(qk, D, D, B, T), _tok_view(qkv, 2 * D, D, B, T),
                   _tok_view(o, 0, D, B, T), lse, _tok_view(do, 0, D, B, T), H, dq=_tok_view(dqk, 0, D, B, T),
                   dk=_tok_view(dqk, D, D, B, T), dv=_tok_view(dqkv, 2 * D, D, B, T))
        K.qknorm_rope_bwd(qkv, 0, D, dqk, H, B, L, _norm_w(ctx.norms), cs, sn, dqkv, 0, D, dw=_norm_g(ctx.norms),
                          dw_acc=_norm_acc(ctx.norms))
        _norm_done(ctx.norms, None)
        return (dqkv, None, None, None) + (None,) * (len(ctx.needs_input_grad) - 4)


class SingleMixFn(torch.autograd.Function):
    """single block: u = [q | k | v | mlp_pre] [T*B, 7D] -> cat = [attention(RMSNorm+RoPE q/k, v) |
    GELU_tanh(mlp_pre)] [T*B, 5D], the proj_out operand (no torch.cat)."""

    @staticmethod
    def forward(ctx, u, geo, norms, rope, *params):
        T, B, H, L = geo
        D = H * 128
        cs, sn = rope
        qk = K.qknorm_rope_fwd(u, 0, D, H, B, 0, _norm_w(norms), cs, sn)
        cat = torch.empty((T * B, 5 * D), dtype=torch.bfloat16, device=u.device)
        _, lse = K.attn_fwd(_tok_view(qk, 0, D, B, T), _tok_view(qk, D, D, B, T), _tok_view(u, 2 * D, D, B, T), H,
                            out=_tok_view(cat, 0, D, B, T))
        K.gelu_tanh_fwd(u[:, 3 * D:], out=cat[:, D:])
        ctx.save_for_backward(u, qk, cat, lse)
        ctx.geo, ctx.norms, ctx.rope = geo, norms, rope
        return cat

    @staticmethod
    def backward(ctx, dcat):
        u, qk, cat, lse = ctx.saved_tensors
        T, B, H, L = ctx.geo
        D = H * 128
        cs, sn = ctx.rope
        if dcat.stride(1) != 1 or dcat.stride(0) % 8:
            dcat = dcat.contiguous()
        du = torch.empty_like(u)
        dqk = torch.empty_like(qk)
        K.attn_bwd(_tok_view(qk, 0, D, B, T), _tok_view(qk, D, D, B, T), _tok_view(u, 2 * D, D, B, T),
                   _tok_view(cat, 0, D, B, T), lse, _tok_view(dcat, 0, D, B, T), H, dq=_tok_view(dqk, 0, D, B, T),
                   dk=_tok_view(dqk, D, D, B, T), dv=_tok_view(du, 2 * D, D, B, T))
        K.gelu_tanh_bwd(u[:, 3 * D:], dcat[:, D:], dx=du[:, 3 * D:])
        K.qknorm_rope_bwd(u, 0, D, dqk, H, B, 0, _norm_w(ctx.norms), cs, sn, du, 0, D, dw=_norm_g(ctx.norms),
                          dw_acc=_norm_acc(ctx.norms))
        _norm_done(ctx.norms, None)
        return (du, None, None, None) + (None,) * (len(ctx.needs_input_grad) - 4)


class GeluTanhFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return K.gelu_tanh_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return K.gelu_tanh_bwd(x, dy.contiguous() if dy.stride(1) != 1 else dy)


class UnpackFn(torch.autograd.Function):
    """FluxModel.unpack_latents: tokens [N*B, 4C] -> NHWC [B, h, w, C]; backward = pack."""

    @staticmethod
    def forward(ctx, tok, B, h, w, C):
        ctx.shape = (B, h, w, C)
        return K.flux_unpack(tok.contiguous(), B, h, w, C)

    @staticmethod
    def backward(ctx, d):
        return K.flux_pack(d.contiguous()), None, None, None, None
