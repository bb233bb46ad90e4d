"""CPU fp32 restatement of diffusers FluxTransformer2DModel + FluxModel.pack/unpack latents, with
diffusers parameter names.  TEST INFRASTRUCTURE ONLY (oracle/__init__.py).

The reference calls it at modules/modelSetup/BaseFluxSetup.py:289-299 (model.transformer(hidden_states=packed,
timestep=t/1000, guidance, pooled_projections, encoder_hidden_states, txt_ids, img_ids)); the pack / unpack /
image-id helpers are modules/model/FluxModel.py:300-344.  diffusers@5873377 is not in this image, so the
network is restated from FLUX.1's published architecture (19 double-stream MMDiT blocks, 38 single-stream
blocks, D = 3072 = 24 heads x 128, RMSNorm q/k, RoPE over (16, 56, 56) id axes, adaLN-Zero modulation,
GELU(tanh) MLPs): PARITY UNPINNED (no reference test or fixture pins the transformer numerics).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class FluxConfig:
    in_channels: int = 64
    num_layers: int = 19
    num_single_layers: int = 38
    attention_head_dim: int = 128
    num_attention_heads: int = 24
    joint_attention_dim: int = 4096
    pooled_projection_dim: int = 768
    guidance_embeds: bool = True
    axes_dims_rope: tuple = (16, 56, 56)
    theta: float = 10000.0

    @property
    def inner_dim(self) -> int:
        return self.num_attention_heads * self.attention_head_dim


def flux_dev_config() -> FluxConfig:
    return FluxConfig()


def tiny_flux_config() -> FluxConfig:
    return FluxConfig(num_layers=2, num_single_layers=2, num_attention_heads=2, joint_attention_dim=64,
                      pooled_projection_dim=32)


def timestep_embedding(t: torch.Tensor, dim: int) -> torch.Tensor:
    """diffusers get_timestep_embedding(flip_sin_to_cos=True, downscale_freq_shift=0)."""
    half = dim // 2
    exponent = -math.log(10000) * torch.arange(half, dtype=torch.float32) / half
    emb = t[:, None].float() * torch.exp(exponent)[None]
    return torch.cat([torch.cos(emb), torch.sin(emb)], dim=-1)


def rope_tables(ids: torch.Tensor, axes_dims, theta=10000.0):
    """FluxPosEmbed: per id axis get_1d_rotary_pos_embed(use_real, repeat_interleave_real, float64)."""
    cos_l, sin_l = [], []
    pos = ids.double()
    for i, d in enumerate(axes_dims):
        freqs = 1.0 / (theta ** (torch.arange(0, d, 2, dtype=torch.float64)[: d // 2] / d))
        f = torch.outer(pos[:, i], freqs)
        cos_l.append(f.cos().repeat_interleave(2, dim=1).float())
        sin_l.append(f.sin().repeat_interleave(2, dim=1).float())
    return torch.cat(cos_l, -1), torch.cat(sin_l, -1)


def apply_rotary_emb(x, cos, sin):
    """x [B, H, S, D]; interleaved real / imaginary pairs (use_real_unbind_dim=-1)."""
    xr, xi = x.reshape(*x.shape[:-1], -1, 2).unbind(-1)
    rot = torch.stack([-xi, xr], dim=-1).flatten(3)
    return x * cos[None, None] + rot * sin[None, None]


class RMSNorm(nn.Module):
    def __init__(self, dim, eps=1e-6):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + self.eps) * self.weight


class TimestepEmbedding(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.linear_1 = nn.Linear(cin, cout)
        self.linear_2 = nn.Linear(cout, cout)

    def forward(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


class CombinedTimestepGuidanceTextProjEmbeddings(nn.Module):
    def __init__(self, dim, pooled_dim, guidance):
        super().__init__()
        self.timestep_embedder = TimestepEmbedding(256, dim)
        if guidance:
            self.guidance_embedder = TimestepEmbedding(256, dim)
        self.text_embedder = TimestepEmbedding(pooled_dim, dim)   # PixArtAlphaTextProjection(act_fn="silu")
        self.guidance = guidance

    def forward(self, timestep, guidance, pooled):
        emb = self.timestep_embedder(timestep_embedding(timestep, 256))
        if self.guidance:
            emb = emb + self.guidance_embedder(timestep_embedding(guidance, 256))
        return emb + self.text_embedder(pooled)


class AdaLNLinear(nn.Module):
    """AdaLayerNormZero / ...Single / ...Continuous: the modulation Linear over silu(temb)."""

    def __init__(self, dim, n):
        super().__init__()
        self.linear = nn.Linear(dim, n * dim)
        self.n = n

    def forward(self, temb):
        return self.linear(F.silu(temb)).chunk(self.n, dim=1)


def _ln(x):
    return F.layer_norm(x, (x.shape[-1],), eps=1e-6)


class FeedForward(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.net = nn.ModuleList([nn.Module(), nn.Dropout(0.0), nn.Linear(4 * dim, dim)])
        self.net[0].proj = nn.Linear(dim, 4 * dim)

    def forward(self, x):
        return self.net[2](F.gelu(self.net[0].proj(x), approximate="tanh"))


def _heads(x, H):
    B, S, C = x.shape
    return x.view(B, S, H, C // H).transpose(1, 2)


class DoubleAttention(nn.Module):
    def __init__(self, dim, H):
        super().__init__()
        self.H = H
        hd = dim // H
        self.to_q, self.to_k, self.to_v = nn.Linear(dim, dim), nn.Linear(dim, dim), nn.Linear(dim, dim)
        self.norm_q, self.norm_k = RMSNorm(hd), RMSNorm(hd)
        self.add_q_proj, self.add_k_proj, self.add_v_proj = nn.Linear(dim, dim), nn.Linear(dim, dim), nn.Linear(dim, dim)
        self.norm_added_q, self.norm_added_k = RMSNorm(hd), RMSNorm(hd)
        self.to_out = nn.ModuleList([nn.Linear(dim, dim)])
        self.to_add_out = nn.Linear(dim, dim)

    def forward(self, x, ctx, cos, sin):
        H, L = self.H, ctx.shape[1]
        q = self.norm_q(_heads(self.to_q(x), H))
        k = self.norm_k(_heads(self.to_k(x), H))
        v = _heads(self.to_v(x), H)
        cq = self.norm_added_q(_heads(self.add_q_proj(ctx), H))
        ck = self.norm_added_k(_heads(self.add_k_proj(ctx), H))
        cv = _heads(self.add_v_proj(ctx), H)
        q, k, v = torch.cat([cq, q], 2), torch.cat([ck, k], 2), torch.cat([cv, v], 2)
        q, k = apply_rotary_emb(q, cos, sin), apply_rotary_emb(k, cos, sin)
        o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).flatten(2)
        return self.to_out[0](o[:, L:]), self.to_add_out(o[:, :L])


class SingleAttention(nn.Module):
    def __init__(self, dim, H):
        super().__init__()
        self.H = H
        hd = dim // H
        self.to_q, self.to_k, self.to_v = nn.Linear(dim, dim), nn.Linear(dim, dim), nn.Linear(dim, dim)
        self.norm_q, self.norm_k = RMSNorm(hd), RMSNorm(hd)

    def forward(self, x, cos, sin):
        H = self.H
        q = apply_rotary_emb(self.norm_q(_heads(self.to_q(x), H)), cos, sin)
        k = apply_rotary_emb(self.norm_k(_heads(self.to_k(x), H)), cos, sin)
        v = _heads(self.to_v(x), H)
        return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).flatten(2)


class FluxTransformerBlock(nn.Module):
    def __init__(self, dim, H):
        super().__init__()
        self.norm1 = AdaLNLinear(dim, 6)
        self.norm1_context = AdaLNLinear(dim, 6)
        self.attn = DoubleAttention(dim, H)
        self.ff = FeedForward(dim)
        self.ff_context = FeedForward(dim)

    def forward(self, x, ctx, temb, cos, sin):
        sh, sc, g, sh2, sc2, g2 = self.norm1(temb)
        csh, csc, cg, csh2, csc2, cg2 = self.norm1_context(temb)
        nx = _ln(x) * (1 + sc[:, None]) + sh[:, None]
        nc = _ln(ctx) * (1 + csc[:, None]) + csh[:, None]
        a, ca = self.attn(nx, nc, cos, sin)
        x = x + g[:, None] * a
        x = x + g2[:, None] * self.ff(_ln(x) * (1 + sc2[:, None]) + sh2[:, None])
        ctx = ctx + cg[:, None] * ca
        ctx = ctx + cg2[:, None] * self.ff_context(_ln(ctx) * (1 + csc2[:, None]) + csh2[:, None])
        return ctx, x


class FluxSingleTransformerBlock(nn.Module):
    def __init__(self, dim, H):
        super().__init__()
        self.norm = AdaLNLinear(dim, 3)
        self.proj_mlp = nn.Linear(dim, 4 * dim)
        self.proj_out = nn.Linear(5 * dim, dim)
        self.attn = SingleAttention(dim, H)

    def forward(self, x, temb, cos, sin):
        sh, sc, g = self.norm(temb)
        n = _ln(x) * (1 + sc[:, None]) + sh[:, None]
        mlp = F.gelu(self.proj_mlp(n), approximate="tanh")
        a = self.attn(n, cos, sin)
        return x + g[:, None] * self.proj_out(torch.cat([a, mlp], dim=2))


class FluxTransformer2DModel(nn.Module):
    def __init__(self, cfg: FluxConfig):
        super().__init__()
        self.cfg = cfg
        D = cfg.inner_dim
        self.time_text_embed = CombinedTimestepGuidanceTextProjEmbeddings(D, cfg.pooled_projection_dim,
                                                                         cfg.guidance_embeds)
        self.context_embedder = nn.Linear(cfg.joint_attention_dim, D)
        self.x_embedder = nn.Linear(cfg.in_channels, D)
        self.transformer_blocks = nn.ModuleList([FluxTransformerBlock(D, cfg.num_attention_heads)
                                                 for _ in range(cfg.num_layers)])
        self.single_transformer_blocks = nn.ModuleList([FluxSingleTransformerBlock(D, cfg.num_attention_heads)
                                                        for _ in range(cfg.num_single_layers)])
        self.norm_out = nn.Module()
        self.norm_out.linear = nn.Linear(D, 2 * D)
        self.proj_out = nn.Linear(D, cfg.in_channels)

    def forward(self, hidden_states, timestep, guidance, pooled_projections, encoder_hidden_states, txt_ids, img_ids):
        """diffusers forward: timestep / guidance are pre-scaled by 1000 inside (as the reference passes t/1000).
        The transformer runs them through the bf16 train dtype first: t_eff = bf16(bf16(t) * 1000)."""
        cfg = self.cfg
        t = (timestep.to(torch.bfloat16) * 1000).float()
        g = (guidance.to(torch.bfloat16) * 1000).float() if guidance is not None else None
        temb = self.time_text_embed(t, g, pooled_projections)
        x = self.x_embedder(hidden_states)
        ctx = self.context_embedder(encoder_hidden_states)
        cos, sin = rope_tables(torch.cat([txt_ids, img_ids], 0), cfg.axes_dims_rope, cfg.theta)
        for blk in self.transformer_blocks:
            ctx, x = blk(x, ctx, temb, cos, sin)
        h = torch.cat([ctx, x], 1)
        for blk in self.single_transformer_blocks:
            h = blk(h, temb, cos, sin)
        x = h[:, ctx.shape[1]:]
        scale, shift = self.norm_out.linear(F.silu(temb)).chunk(2, dim=1)
        x = _ln(x) * (1 + scale[:, None]) + shift[:, None]
        return self.proj_out(x)


# ---- FluxModel helpers (modules/model/FluxModel.py:300-344) ----
def prepare_latent_image_ids(height, width):
    ids = torch.zeros(height // 2, width // 2, 3)
    ids[..., 1] = ids[..., 1] + torch.arange(height // 2)[:, None]
    ids[..., 2] = ids[..., 2] + torch.arange(width // 2)[None, :]
    return ids.reshape(-1, 3)


def pack_latents(latents):
    B, C, H, W = latents.shape
    x = latents.view(B, C, H // 2, 2, W // 2, 2).permute(0, 2, 4, 1, 3, 5)
    return x.reshape(B, (H // 2) * (W // 2), C * 4)


def unpack_latents(latents, height, width):
    B, P, C = latents.shape
    x = latents.view(B, height // 2, width // 2, C // 4, 2, 2).permute(0, 3, 1, 4, 2, 5)
    return x.reshape(B, C // 4, height, width)
