"""CPU fp32 restatement of diffusers AutoencoderKL.encode(...).latent_dist.mean (the encoder half +
quant_conv + DiagonalGaussianDistribution mean), NCHW, diffusers parameter names.
TEST INFRASTRUCTURE ONLY (oracle/__init__.py).

The reference runs it through mgds EncodeVAE + SampleVAEDistribution(mode='mean') at
modules/dataLoader/StableDiffusionXLBaseDataLoader.py:65-100 (RescaleImageChannels 0..1 -> -1..1 first).
diffusers@5873377 and mgds@11ff4aa are not in this image; the graph is restated from the ddconfig
the reference pins in resources/model_config/stable_diffusion_xl/sd_xl_base.yaml (ch 128,
ch_mult [1,2,4,4], num_res_blocks 2, z_channels 4, double_z, attn only in the mid block).
FLUX.1 (FluxBaseDataLoader.py:70-71): 16 latent channels and no quant_conv (cfg.use_quant_conv False): the
mean is conv_out's first 16 channels.
PARITY UNPINNED: no reference test or fixture pins the VAE numerics.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class ResnetBlock2D(nn.Module):
    """diffusers ResnetBlock2D with temb_channels=None (VAE), GroupNorm eps 1e-6."""

    def __init__(self, cin, cout, groups, eps):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, cin, eps)
        self.conv1 = nn.Conv2d(cin, cout, 3, 1, 1)
        self.norm2 = nn.GroupNorm(groups, cout, eps)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1)
        self.conv_shortcut = nn.Conv2d(cin, cout, 1) if cin != cout else None

    def forward(self, x):
        h = self.conv1(F.silu(self.norm1(x)))
        h = self.conv2(F.silu(self.norm2(h)))
        if self.conv_shortcut is not None:
            x = self.conv_shortcut(x)
        return x + h


class Downsample2D(nn.Module):
    """padding=0 variant: F.pad(x, (0, 1, 0, 1)) then 3x3 stride-2 conv."""

    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 2, 0)

    def forward(self, x):
        return self.conv(F.pad(x, (0, 1, 0, 1)))


class VAEAttention(nn.Module):
    """single-head self-attention with GroupNorm, biased projections and the residual add."""

    def __init__(self, c, groups, eps):
        super().__init__()
        self.group_norm = nn.GroupNorm(groups, c, eps)
        self.to_q, self.to_k, self.to_v = nn.Linear(c, c), nn.Linear(c, c), nn.Linear(c, c)
        self.to_out = nn.ModuleList([nn.Linear(c, c)])

    def forward(self, x):
        B, C, H, W = x.shape
        h = self.group_norm(x).view(B, C, H * W).transpose(1, 2)
        q, k, v = self.to_q(h)[:, None], self.to_k(h)[:, None], self.to_v(h)[:, None]
        o = F.scaled_dot_product_attention(q, k, v)[:, 0]
        o = self.to_out[0](o)
        return o.transpose(1, 2).reshape(B, C, H, W) + x


class DownEncoderBlock2D(nn.Module):
    def __init__(self, cin, cout, layers, add_down, groups, eps):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, groups, eps) for i in range(layers)])
        if add_down:
            self.downsamplers = nn.ModuleList([Downsample2D(cout)])
        self.add_down = add_down

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.add_down:
            x = self.downsamplers[0](x)
        return x


class MidBlock(nn.Module):
    def __init__(self, c, groups, eps):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(c, c, groups, eps) for _ in range(2)])
        self.attentions = nn.ModuleList([VAEAttention(c, groups, eps)])

    def forward(self, x):
        return self.resnets[1](self.attentions[0](self.resnets[0](x)))


class Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        ch = cfg.block_out_channels
        g, eps = cfg.norm_num_groups, cfg.norm_eps
        self.conv_in = nn.Conv2d(cfg.in_channels, ch[0], 3, 1, 1)
        self.down_blocks = nn.ModuleList()
        cin = ch[0]
        for i, c in enumerate(ch):
            self.down_blocks.append(DownEncoderBlock2D(cin, c, cfg.layers_per_block, i < len(ch) - 1, g, eps))
            cin = c
        self.mid_block = MidBlock(ch[-1], g, eps)
        self.conv_norm_out = nn.GroupNorm(g, ch[-1], eps)
        self.conv_out = nn.Conv2d(ch[-1], 2 * cfg.latent_channels, 3, 1, 1)

    def forward(self, x):
        x = self.conv_in(x)
        for b in self.down_blocks:
            x = b(x)
        x = self.mid_block(x)
        return self.conv_out(F.silu(self.conv_norm_out(x)))


class AutoencoderKLEncoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.encoder = Encoder(cfg)
        q = getattr(cfg, "use_quant_conv", True)
        self.quant_conv = nn.Conv2d(2 * cfg.latent_channels, 2 * cfg.latent_channels, 1) if q else None

    def moments(self, x):
        """x: rescaled image in [-1, 1] -> the DiagonalGaussianDistribution parameters"""
        h = self.encoder(x)
        return self.quant_conv(h) if self.quant_conv is not None else h

    def forward(self, images01):
        """images in [0, 1] NCHW -> latent_dist.mean NCHW (RescaleImageChannels + encode + mean)."""
        return self.moments(images01 * 2.0 - 1.0)[:, :self.cfg.latent_channels]
