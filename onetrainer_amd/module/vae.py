"""AutoencoderKL encoder (latent caching) on the HIP kernels: NHWC bf16, frozen flat store,
diffusers parameter names.

Drop-in for what the reference's data pipeline runs once per image variation before the steps
(SURVEY.md §8(a) a18): mgds EncodeVAE + SampleVAEDistribution(mode='mean') wired at
modules/dataLoader/StableDiffusionXLBaseDataLoader.py:65-100 (RescaleImageChannels 0..1 -> -1..1,
vae.encode(image).latent_dist, mean).  Architecture: diffusers AutoencoderKL Encoder with the
ddconfig of resources/model_config/stable_diffusion_xl/sd_xl_base.yaml (ch 128, ch_mult
[1, 2, 4, 4], num_res_blocks 2, z_channels 4, double_z) -- the SD 1.5 VAE has the same encoder.

Encoder graph (forward only; nothing is trained):
  conv_in 3->128 | 4 x DownEncoderBlock2D (2 x ResnetBlock2D, GN eps 1e-6, no time embedding;
  Downsample2D = F.pad(0,1,0,1) + 3x3 stride-2 conv on all but the last) | mid: ResnetBlock2D,
  single-head self-attention (GroupNorm, to_q/k/v/out with bias, residual), ResnetBlock2D |
  GN + SiLU, conv_out 512->8 | quant_conv 1x1 8->8 | mean = channels [0, 4).
FLUX.1's AutoencoderKL (flux_vae_config, FluxBaseDataLoader.py:70-71 + BaseFluxSetup.py:229-230) has the same
encoder with 16 latent channels (conv_out 512->32) and no quant_conv: mean = conv_out channels [0, 16); the
setup applies (latent - shift_factor) * scaling_factor.
Kernels: implicit-GEMM convs (stride 2 + one-sided zero padding through the conv gather's range
check), GroupNorm(+SiLU), fused q|k|v Linear, the materialized single-head attention (512-wide
head: batched MFMA GEMMs + row softmax), and the quant_conv mean rows as one fp32-out GEMM.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .. import kernels as K
from .param_store import FlatParamStore

BF16 = torch.bfloat16
PAD_IN = 8    # conv_in input channels held (RGB zero-padded to one 16-byte chunk)


@dataclass
class VAEConfig:
    in_channels: int = 3
    block_out_channels: tuple = (128, 256, 512, 512)
    layers_per_block: int = 2
    latent_channels: int = 4
    norm_num_groups: int = 32
    norm_eps: float = 1e-6
    scaling_factor: float = 0.13025
    shift_factor: float = 0.0
    use_quant_conv: bool = True


def sdxl_vae_config() -> VAEConfig:
    return VAEConfig()


def sd15_vae_config() -> VAEConfig:
    return VAEConfig(scaling_factor=0.18215)


def flux_vae_config() -> VAEConfig:
    """black-forest-labs/FLUX.1-dev vae/config.json: latent_channels 16, use_quant_conv false,
    scaling_factor 0.3611, shift_factor 0.1159 (the encoder otherwise equals SDXL's)."""
    return VAEConfig(latent_channels=16, scaling_factor=0.3611, shift_factor=0.1159, use_quant_conv=False)


def tiny_vae_config(latent_channels: int = 4, use_quant_conv: bool = True) -> VAEConfig:
    """test size; 160 mid channels -> a 160-wide single head (materialized attention path)."""
    return VAEConfig(block_out_channels=(64, 160), layers_per_block=1, latent_channels=latent_channels,
                     use_quant_conv=use_quant_conv)


def _conv(p, cin, cout, k=3):
    return [(p + ".weight", (cout, cin, k, k), "conv", cin * k * k), (p + ".bias", (cout,), "bias", cin * k * k)]


def _norm(p, c):
    return [(p + ".weight", (c,), "norm_w", 0), (p + ".bias", (c,), "norm_b", 0)]


def _resnet(p, cin, cout):
    s = _norm(p + ".norm1", cin) + _conv(p + ".conv1", cin, cout) + _norm(p + ".norm2", cout)
    s += _conv(p + ".conv2", cout, cout)
    if cin != cout:
        s += _conv(p + ".conv_shortcut", cin, cout, 1)
    return s


def vae_encoder_specs(cfg: VAEConfig):
    """(name, diffusers shape, kind, fan_in) in execution order; q|k|v weights then q|k|v biases
    are adjacent so the fused projection is one view."""
    ch = cfg.block_out_channels
    s = _conv("encoder.conv_in", cfg.in_channels, ch[0])
    cin = ch[0]
    for i, c in enumerate(ch):
        for j in range(cfg.layers_per_block):
            s += _resnet(f"encoder.down_blocks.{i}.resnets.{j}", cin if j == 0 else c, c)
        if i < len(ch) - 1:
            s += _conv(f"encoder.down_blocks.{i}.downsamplers.0.conv", c, c)
        cin = c
    c = ch[-1]
    a = "encoder.mid_block.attentions.0"
    s += _resnet("encoder.mid_block.resnets.0", c, c)
    s += _norm(a + ".group_norm", c)
    s += [(f"{a}.to_{x}.weight", (c, c), "linear", c) for x in "qkv"]
    s += [(f"{a}.to_{x}.bias", (c,), "bias", c) for x in "qkv"]
    s += [(a + ".to_out.0.weight", (c, c), "linear", c), (a + ".to_out.0.bias", (c,), "bias", c)]
    s += _resnet("encoder.mid_block.resnets.1", c, c)
    s += _norm("encoder.conv_norm_out", c) + _conv("encoder.conv_out", c, 2 * cfg.latent_channels)
    if cfg.use_quant_conv:
        s += _conv("quant_conv", 2 * cfg.latent_channels, 2 * cfg.latent_channels, 1)
    return s


def _store_shape(name, shape, kind):
    if kind == "conv":
        co, ci, kh, kw = shape
        if name == "encoder.conv_in.weight":
            ci = PAD_IN
        return (co, ci) if kh == 1 else (co, kh, kw, ci)
    return shape


def flops_per_image(cfg: VAEConfig, h: int, w: int) -> float:
    """analytic encoder FLOPs (2 x MACs; norms / softmax excluded) at image size h x w."""
    macs = h * w * cfg.in_channels * cfg.block_out_channels[0] * 9
    ch = cfg.block_out_channels
    cin = ch[0]
    hw = h * w
    for i, c in enumerate(ch):
        for j in range(cfg.layers_per_block):
            ci = cin if j == 0 else c
            macs += hw * ci * c * 9 + hw * c * c * 9 + (hw * ci * c if ci != c else 0)
        if i < len(ch) - 1:
            hw //= 4
            macs += hw * c * c * 9
        cin = c
    c = ch[-1]
    macs += 2 * (2 * hw * c * c * 9) + 4 * hw * c * c + 2 * hw * hw * c
    lc = 2 * cfg.latent_channels
    macs += hw * c * lc * 9 + (hw * lc * lc if cfg.use_quant_conv else 0)
    return 2.0 * macs


class AutoencoderKLEncoder:
    """VAE encoder for latent caching; weights in a frozen FlatParamStore (bf16)."""

    def __init__(self, cfg: VAEConfig, device, dtype=BF16, seed: int | None = 0):
        self.cfg = cfg
        self.device = torch.device(device)
        self.specs = vae_encoder_specs(cfg)
        self.store = FlatParamStore([(n, _store_shape(n, sh, k), "vae") for n, sh, k, _ in self.specs], dtype,
                                    self.device, trainable=False)
        self.config = {"scaling_factor": cfg.scaling_factor, "shift_factor": cfg.shift_factor}
        if seed is not None:
            self.init_weights(seed)

    # ----- parameters ---------------------------------------------------------------------------
    def init_weights(self, seed: int):
        g = torch.Generator(device=self.device).manual_seed(seed)
        with torch.no_grad():
            for name, shape, kind, fan_in in self.specs:
                if kind in ("linear", "conv", "bias"):
                    b = 1.0 / math.sqrt(fan_in)
                    self._assign(name, (torch.rand(shape, generator=g, device=self.device) * 2 - 1) * b, kind)
                elif kind == "norm_w":
                    self.store.params[name].fill_(1.0)
                else:
                    self.store.params[name].zero_()

    def _assign(self, name, v, kind):
        p = self.store.params[name]
        if kind == "conv":
            v = v.permute(0, 2, 3, 1) if v.shape[2] > 1 else v.reshape(v.shape[0], v.shape[1])
            if name == "encoder.conv_in.weight":
                v = torch.nn.functional.pad(v, (0, PAD_IN - v.shape[-1]))
        p.data.copy_(v.to(p.dtype))

    def num_parameters(self) -> int:
        return sum(math.prod(sh) for _, sh, _, _ in self.specs)

    def state_dict(self, dtype=None):
        out = {}
        for name, shape, kind, _ in self.specs:
            v = self.store.params[name].detach()
            if kind == "conv":
                v = v.reshape(v.shape[0], v.shape[1], 1, 1) if v.dim() == 2 else v.permute(0, 3, 1, 2)
                v = v[:, :shape[1]]
            out[name] = v.to(dtype or v.dtype).contiguous()
        return out

    def load_state_dict(self, sd):
        """diffusers AutoencoderKL keys (encoder.* and quant_conv.* when the config has one; decoder keys are
        ignored)."""
        with torch.no_grad():
            for name, shape, kind, _ in self.specs:
                if tuple(sd[name].shape) != tuple(shape):
                    raise ValueError(f"{name}: shape {tuple(sd[name].shape)} != {shape}")
                self._assign(name, sd[name].to(self.device, torch.float32), kind)

    def W(self, name):
        return self.store.params[name].data

    # ----- blocks -------------------------------------------------------------------------------
    def _gn(self, x, p, silu):
        y, _ = K.groupnorm_fwd(x, self.W(p + ".weight"), self.W(p + ".bias"), self.cfg.norm_num_groups,
                               self.cfg.norm_eps, silu)
        return y

    def _resnet(self, x, p):
        h = self._gn(x, p + ".norm1", True)
        h = K.conv2d(h, self.W(p + ".conv1.weight"), bias=self.W(p + ".conv1.bias"))
        h = self._gn(h, p + ".norm2", True)
        sc = x
        if (p + ".conv_shortcut.weight") in self.store.slots:
            N, H, W_, C = x.shape
            sc = K.linear(x.view(-1, C), self.W(p + ".conv_shortcut.weight"),
                          bias=self.W(p + ".conv_shortcut.bias")).view(N, H, W_, -1)
        return K.conv2d(h, self.W(p + ".conv2.weight"), bias=self.W(p + ".conv2.bias"), residual=sc)

    def _attention(self, x, p):
        N, H, W_, C = x.shape
        h = self._gn(x, p + ".group_norm", False).view(N, H * W_, C)
        wqkv = self.store.view([f"{p}.to_{c}.weight" for c in "qkv"], (3 * C, C))
        bqkv = self.store.view([f"{p}.to_{c}.bias" for c in "qkv"], (3 * C,))
        qkv = K.linear(h.view(-1, C), wqkv, bias=bqkv).view(N, H * W_, 3 * C)
        o, _ = K.attn_fwd(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], 1)
        out = K.linear(o.view(-1, C), self.W(p + ".to_out.0.weight"), bias=self.W(p + ".to_out.0.bias"),
                       residual=x.view(-1, C))
        return out.view(N, H, W_, C)

    # ----- encode -------------------------------------------------------------------------------
    @torch.no_grad()
    def encode_nhwc(self, x):
        """x: [B, H, W, 8] bf16 in [-1, 1] (channels >= 3 zero) -> latent mean [B, H/8, W/8, L] fp32."""
        cfg = self.cfg
        ch = cfg.block_out_channels
        K._req(x.shape[1] % (1 << (len(ch) - 1)) == 0 and x.shape[2] % (1 << (len(ch) - 1)) == 0,
               "image size must be a multiple of the VAE downsampling factor")
        h = K.conv2d(x, self.W("encoder.conv_in.weight"), bias=self.W("encoder.conv_in.bias"))
        for i, c in enumerate(ch):
            for j in range(cfg.layers_per_block):
                h = self._resnet(h, f"encoder.down_blocks.{i}.resnets.{j}")
            if i < len(ch) - 1:
                p = f"encoder.down_blocks.{i}.downsamplers.0.conv"
                N, H, W_, _ = h.shape
                h = K.conv2d(h, self.W(p + ".weight"), bias=self.W(p + ".bias"), stride=2, pad=0,
                             out_hw=(H // 2, W_ // 2))
        h = self._resnet(h, "encoder.mid_block.resnets.0")
        h = self._attention(h, "encoder.mid_block.attentions.0")
        h = self._resnet(h, "encoder.mid_block.resnets.1")
        h = self._gn(h, "encoder.conv_norm_out", True)
        L = cfg.latent_channels
        if not cfg.use_quant_conv:
            # DiagonalGaussianDistribution(conv_out(h)).mean: only conv_out's first L output channels (the stored
            # weight's first L rows), in the reference's autocast dtype
            mean = K.conv2d(h, self.W("encoder.conv_out.weight")[:L], bias=self.W("encoder.conv_out.bias")[:L])
            return mean.float()
        h = K.conv2d(h, self.W("encoder.conv_out.weight"), bias=self.W("encoder.conv_out.bias"))
        N, H, W_, C2 = h.shape
        # DiagonalGaussianDistribution(quant_conv(h)).mean: only the first L quant_conv rows
        mean = K.linear(h.view(-1, C2), self.W("quant_conv.weight")[:L], bias=self.W("quant_conv.bias")[:L],
                        out_dtype=torch.float32)
        return mean.view(N, H, W_, L)

    def encode(self, images):
        """images: [B, 3, H, W] fp32 in [0, 1] (mgds image range) -> latent mean NHWC fp32."""
        return self.encode_nhwc(K.image_to_nhwc(images.contiguous(), 2.0, -1.0, PAD_IN))

    __call__ = encode
