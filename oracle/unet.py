"""CPU fp32 restatement of diffusers UNet2DConditionModel (SD 1.5 / SDXL), NCHW, diffusers
parameter names.  TEST INFRASTRUCTURE ONLY (oracle/__init__.py).

The reference calls diffusers@5873377 (requirements-global.txt:22) at
modules/modelSetup/BaseStableDiffusionXLSetup.py:268-273 and BaseStableDiffusionSetup.py:202-206;
diffusers is not in this image, so the network is restated from the architecture the reference
pins in-tree:
  resources/model_config/stable_diffusion_xl/sd_xl_base.yaml:19-37   (SDXL: 320/640/1280, depth [0,2,10],
                                                                       head dim 64, ctx 2048, adm 2816)
  resources/model_config/stable_diffusion/v1-inference.yaml:29-44     (SD1.5: 320x[1,2,4,4], 8 heads, ctx 768)
  modules/util/convert/convert_sdxl_diffusers_to_ckpt.py:8-81          (module graph / parameter names)
PARITY UNPINNED: no reference test pins the network numerics; parameter counts reproduce the
known totals (SDXL 2,567,463,684; SD1.5 859,520,964 -- tests/test_unet_spec.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class UNetConfig:
    in_channels: int = 4
    out_channels: int = 4
    block_out_channels: tuple = (320, 640, 1280)
    down_block_types: tuple = ("DownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D")
    up_block_types: tuple = ("CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "UpBlock2D")
    layers_per_block: int = 2
    transformer_layers_per_block: tuple = (1, 2, 10)
    head_dim: int | None = 64            # SDXL: fixed head dim 64 (heads = C / 64)
    num_heads: int | None = None         # SD1.5: fixed 8 heads (head dim = C / 8)
    cross_attention_dim: int = 2048
    use_linear_projection: bool = True
    addition_embed: bool = True          # SDXL "text_time" add embedding
    addition_time_embed_dim: int = 256
    projection_class_embeddings_input_dim: int = 2816
    norm_num_groups: int = 32
    norm_eps: float = 1e-5
    temb_dim: int = field(default=0)

    def __post_init__(self):
        if not self.temb_dim:
            self.temb_dim = self.block_out_channels[0] * 4

    def heads(self, c: int) -> int:
        return c // self.head_dim if self.head_dim else self.num_heads


def sdxl_config() -> UNetConfig:
    return UNetConfig()


def sd15_config() -> UNetConfig:
    return UNetConfig(block_out_channels=(320, 640, 1280, 1280),
                      down_block_types=("CrossAttnDownBlock2D",) * 3 + ("DownBlock2D",),
                      up_block_types=("UpBlock2D",) + ("CrossAttnUpBlock2D",) * 3,
                      transformer_layers_per_block=(1, 1, 1, 1), head_dim=None, num_heads=8,
                      cross_attention_dim=768, use_linear_projection=False, addition_embed=False)


def tiny_sdxl_config() -> UNetConfig:
    """SDXL-shaped miniature used by parity tests (2 levels, attention at level 1)."""
    return UNetConfig(block_out_channels=(64, 128), down_block_types=("DownBlock2D", "CrossAttnDownBlock2D"),
                      up_block_types=("CrossAttnUpBlock2D", "UpBlock2D"), transformer_layers_per_block=(0, 2),
                      head_dim=64, cross_attention_dim=96, addition_time_embed_dim=32,
                      projection_class_embeddings_input_dim=64 + 6 * 32, norm_num_groups=32)


def timestep_embedding(t: torch.Tensor, dim: int) -> torch.Tensor:
    """diffusers get_timestep_embedding(flip_sin_to_cos=True, downscale_freq_shift=0)."""
    half = dim // 2
    exponent = -math.log(10000) * torch.arange(0, half, dtype=torch.float32, device=t.device)
    exponent = exponent / half
    emb = t[:, None].float() * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    return torch.cat([emb[:, half:], emb[:, :half]], dim=-1)


class TimestepEmbedding(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.linear_1 = nn.Linear(cin, cout)
        self.linear_2 = nn.Linear(cout, cout)

    def forward(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


class ResnetBlock2D(nn.Module):
    def __init__(self, cin, cout, temb, groups, eps):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, cin, eps)
        self.conv1 = nn.Conv2d(cin, cout, 3, 1, 1)
        self.time_emb_proj = nn.Linear(temb, cout)
        self.norm2 = nn.GroupNorm(groups, cout, eps)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1)
        self.conv_shortcut = nn.Conv2d(cin, cout, 1) if cin != cout else None

    def forward(self, x, temb):
        h = self.conv1(F.silu(self.norm1(x)))
        h = h + self.time_emb_proj(F.silu(temb))[:, :, None, None]
        h = self.conv2(F.silu(self.norm2(h)))
        if self.conv_shortcut is not None:
            x = self.conv_shortcut(x)
        return x + h


class Attention(nn.Module):
    def __init__(self, dim, ctx_dim, heads):
        super().__init__()
        self.heads = heads
        self.to_q = nn.Linear(dim, dim, bias=False)
        self.to_k = nn.Linear(ctx_dim, dim, bias=False)
        self.to_v = nn.Linear(ctx_dim, dim, bias=False)
        self.to_out = nn.ModuleList([nn.Linear(dim, dim)])

    def forward(self, x, ctx=None):
        ctx = x if ctx is None else ctx
        B, N, C = x.shape
        q, k, v = self.to_q(x), self.to_k(ctx), self.to_v(ctx)
        sp = lambda t: t.view(B, -1, self.heads, C // self.heads).transpose(1, 2)
        o = F.scaled_dot_product_attention(sp(q), sp(k), sp(v))
        return self.to_out[0](o.transpose(1, 2).reshape(B, N, C))


class GEGLU(nn.Module):
    def __init__(self, dim, inner):
        super().__init__()
        self.proj = nn.Linear(dim, inner * 2)

    def forward(self, x):
        h, gate = self.proj(x).chunk(2, dim=-1)
        return h * F.gelu(gate)


class FeedForward(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.net = nn.ModuleList([GEGLU(dim, 4 * dim), nn.Dropout(0.0), nn.Linear(4 * dim, dim)])

    def forward(self, x):
        for m in self.net:
            x = m(x)
        return x


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim, heads, ctx_dim):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim)
        self.attn1 = Attention(dim, dim, heads)
        self.norm2 = nn.LayerNorm(dim)
        self.attn2 = Attention(dim, ctx_dim, heads)
        self.norm3 = nn.LayerNorm(dim)
        self.ff = FeedForward(dim)

    def forward(self, x, ctx):
        x = self.attn1(self.norm1(x)) + x
        x = self.attn2(self.norm2(x), ctx) + x
        return self.ff(self.norm3(x)) + x


class Transformer2DModel(nn.Module):
    def __init__(self, dim, heads, depth, ctx_dim, linear_proj, groups):
        super().__init__()
        self.linear_proj = linear_proj
        self.norm = nn.GroupNorm(groups, dim, 1e-6)
        self.proj_in = nn.Linear(dim, dim) if linear_proj else nn.Conv2d(dim, dim, 1)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(dim, heads, ctx_dim) for _ in range(depth)])
        self.proj_out = nn.Linear(dim, dim) if linear_proj else nn.Conv2d(dim, dim, 1)

    def forward(self, x, ctx):
        B, C, H, W = x.shape
        res = x
        h = self.norm(x)
        if self.linear_proj:
            h = self.proj_in(h.permute(0, 2, 3, 1).reshape(B, H * W, C))
        else:
            h = self.proj_in(h).permute(0, 2, 3, 1).reshape(B, H * W, C)
        for blk in self.transformer_blocks:
            h = blk(h, ctx)
        if self.linear_proj:
            h = self.proj_out(h).reshape(B, H, W, C).permute(0, 3, 1, 2)
        else:
            h = self.proj_out(h.reshape(B, H, W, C).permute(0, 3, 1, 2))
        return h + res


class Downsample2D(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 2, 1)

    def forward(self, x):
        return self.conv(x)


class Upsample2D(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 1, 1)

    def forward(self, x):
        return self.conv(F.interpolate(x, scale_factor=2.0, mode="nearest"))


class DownBlock(nn.Module):
    def __init__(self, cfg, cin, cout, depth, add_down, cross):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, cfg.temb_dim, cfg.norm_num_groups,
                                                    cfg.norm_eps) for i in range(cfg.layers_per_block)])
        if cross:
            self.attentions = nn.ModuleList([Transformer2DModel(cout, cfg.heads(cout), depth, cfg.cross_attention_dim,
                                                                cfg.use_linear_projection, cfg.norm_num_groups)
                                             for _ in range(cfg.layers_per_block)])
        self.cross = cross
        if add_down:
            self.downsamplers = nn.ModuleList([Downsample2D(cout)])
        self.add_down = add_down

    def forward(self, x, temb, ctx):
        outs = []
        for i, r in enumerate(self.resnets):
            x = r(x, temb)
            if self.cross:
                x = self.attentions[i](x, ctx)
            outs.append(x)
        if self.add_down:
            x = self.downsamplers[0](x)
            outs.append(x)
        return x, outs


class UpBlock(nn.Module):
    def __init__(self, cfg, prev, cout, skip_chs, depth, add_up, cross):
        super().__init__()
        n = cfg.layers_per_block + 1
        self.resnets = nn.ModuleList([ResnetBlock2D((prev if i == 0 else cout) + skip_chs[i], cout, cfg.temb_dim,
                                                    cfg.norm_num_groups, cfg.norm_eps) for i in range(n)])
        if cross:
            self.attentions = nn.ModuleList([Transformer2DModel(cout, cfg.heads(cout), depth, cfg.cross_attention_dim,
                                                                cfg.use_linear_projection, cfg.norm_num_groups)
                                             for _ in range(n)])
        self.cross = cross
        if add_up:
            self.upsamplers = nn.ModuleList([Upsample2D(cout)])
        self.add_up = add_up

    def forward(self, x, skips, temb, ctx):
        for i, r in enumerate(self.resnets):
            x = torch.cat([x, skips.pop()], dim=1)
            x = r(x, temb)
            if self.cross:
                x = self.attentions[i](x, ctx)
        if self.add_up:
            x = self.upsamplers[0](x)
        return x


class MidBlock(nn.Module):
    def __init__(self, cfg, c, depth):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(c, c, cfg.temb_dim, cfg.norm_num_groups, cfg.norm_eps)
                                      for _ in range(2)])
        self.attentions = nn.ModuleList([Transformer2DModel(c, cfg.heads(c), depth, cfg.cross_attention_dim,
                                                            cfg.use_linear_projection, cfg.norm_num_groups)])

    def forward(self, x, temb, ctx):
        x = self.resnets[0](x, temb)
        x = self.attentions[0](x, ctx)
        return self.resnets[1](x, temb)


class UNet2DConditionModel(nn.Module):
    def __init__(self, cfg: UNetConfig):
        super().__init__()
        self.cfg = cfg
        ch = cfg.block_out_channels
        c0 = ch[0]
        self.conv_in = nn.Conv2d(cfg.in_channels, c0, 3, 1, 1)
        self.time_embedding = TimestepEmbedding(c0, cfg.temb_dim)
        if cfg.addition_embed:
            self.add_embedding = TimestepEmbedding(cfg.projection_class_embeddings_input_dim, cfg.temb_dim)
        self.down_blocks = nn.ModuleList()
        skip_chs = [c0]
        cin = c0
        nlev = len(ch)
        for i, bt in enumerate(cfg.down_block_types):
            cout = ch[i]
            blk = DownBlock(cfg, cin, cout, cfg.transformer_layers_per_block[i], i < nlev - 1,
                            bt.startswith("CrossAttn"))
            self.down_blocks.append(blk)
            skip_chs += [cout] * cfg.layers_per_block + ([cout] if i < nlev - 1 else [])
            cin = cout
        self.mid_block = MidBlock(cfg, ch[-1], cfg.transformer_layers_per_block[-1])
        self.up_blocks = nn.ModuleList()
        rev = list(reversed(ch))
        rev_depth = list(reversed(cfg.transformer_layers_per_block))
        prev = ch[-1]
        for i, bt in enumerate(cfg.up_block_types):
            cout = rev[i]
            n = cfg.layers_per_block + 1
            sk = [skip_chs.pop() for _ in range(n)]
            blk = UpBlock(cfg, prev, cout, sk, rev_depth[i], i < nlev - 1, bt.startswith("CrossAttn"))
            self.up_blocks.append(blk)
            prev = cout
        self.conv_norm_out = nn.GroupNorm(cfg.norm_num_groups, c0, cfg.norm_eps)
        self.conv_out = nn.Conv2d(c0, cfg.out_channels, 3, 1, 1)

    def forward(self, sample, timestep, encoder_hidden_states, text_embeds=None, time_ids=None):
        cfg = self.cfg
        B = sample.shape[0]
        t = timestep.expand(B) if timestep.dim() == 1 and timestep.numel() == 1 else timestep
        temb = self.time_embedding(timestep_embedding(t, cfg.block_out_channels[0]).to(sample.dtype))
        if cfg.addition_embed:
            te = timestep_embedding(time_ids.flatten(), cfg.addition_time_embed_dim).reshape(B, -1)
            add = torch.cat([text_embeds, te], dim=-1).to(temb.dtype)
            temb = temb + self.add_embedding(add)
        x = self.conv_in(sample)
        skips = [x]
        for blk in self.down_blocks:
            x, outs = blk(x, temb, encoder_hidden_states)
            skips += outs
        x = self.mid_block(x, temb, encoder_hidden_states)
        for blk in self.up_blocks:
            x = blk(x, skips, temb, encoder_hidden_states)
        return self.conv_out(F.silu(self.conv_norm_out(x)))
