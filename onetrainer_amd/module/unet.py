"""UNet2DConditionModel (SD 1.5 / SDXL) on the HIP kernels: NHWC bf16 activations, flat
parameter store, diffusers parameter names.

Drop-in for the network the reference calls at
  modules/modelSetup/BaseStableDiffusionXLSetup.py:268-273  (model.unet(sample, timestep, ehs, added_cond_kwargs))
  modules/modelSetup/BaseStableDiffusionSetup.py:202-206
Architecture from resources/model_config/stable_diffusion_xl/sd_xl_base.yaml:19-37 and
resources/model_config/stable_diffusion/v1-inference.yaml:29-44; parameter names follow
modules/util/convert/convert_sdxl_diffusers_to_ckpt.py:8-81 so `state_dict()` is a diffusers
UNet state dict (conv weights are held [Cout][kh][kw][Cin] internally and permuted on export).

Layout choices (MI355X-first, not a translation):
  * activations NHWC: a conv's GEMM rows are pixels, and a Transformer2D's proj_in/out are
    Linears over the same [pixels, C] rows (no permutes anywhere);
  * conv_in takes 8 input channels (4 latent + 4 zero) and conv_out emits 8 (4 + 4 zero) so
    every operand row is a whole number of 16-byte chunks;
  * to_q|to_k|to_v (self) and to_k|to_v (cross) are adjacent in the flat store: one GEMM each.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from .. import kernels as K
from . import functional as Fn
from .param_store import FlatParamStore

BF16 = torch.bfloat16


@dataclass
class UNetConfig:
    in_channels: int = 4
    out_channels: int = 4
    block_out_channels: tuple = (320, 640, 1280)
    down_block_types: tuple = ("DownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D")
    up_block_types: tuple = ("CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "UpBlock2D")
    layers_per_block: int = 2
    transformer_layers_per_block: tuple = (1, 2, 10)
    head_dim: int | None = 64
    num_heads: int | None = None
    cross_attention_dim: int = 2048
    use_linear_projection: bool = True
    addition_embed: bool = True
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
    return UNetConfig(block_out_channels=(64, 128), down_block_types=("DownBlock2D", "CrossAttnDownBlock2D"),
                      up_block_types=("CrossAttnUpBlock2D", "UpBlock2D"), transformer_layers_per_block=(0, 2),
                      head_dim=64, cross_attention_dim=96, addition_time_embed_dim=32,
                      projection_class_embeddings_input_dim=64 + 6 * 32, norm_num_groups=32)


def tiny_sd15_config() -> UNetConfig:
    """SD 1.5-shaped (conv proj_in/out, no add-embedding, fixed head count) at test size; 2 heads
    give 80-wide heads (flash kernels) and 160-wide heads (materialized path) like SD 1.5's."""
    return UNetConfig(block_out_channels=(160, 320), down_block_types=("CrossAttnDownBlock2D", "DownBlock2D"),
                      up_block_types=("UpBlock2D", "CrossAttnUpBlock2D"), transformer_layers_per_block=(1, 1),
                      head_dim=None, num_heads=2, cross_attention_dim=96, use_linear_projection=False,
                      addition_embed=False, norm_num_groups=32)


def unet_config_from_diffusers(d: dict) -> UNetConfig:
    """UNet2DConditionModel config.json (what diffusers' from_pretrained builds the architecture from,
    HFModelLoaderMixin.py:61-101) -> UNetConfig.  diffusers' `attention_head_dim` is the head COUNT
    per block (int or list); equal head widths become `head_dim`, else a fixed head count."""
    chans = tuple(d["block_out_channels"])
    n = len(chans)
    heads = d.get("num_attention_heads") or d.get("attention_head_dim", 8)
    heads = list(heads) if isinstance(heads, (list, tuple)) else [heads] * n
    widths = {c // h for c, h in zip(chans, heads)}
    tl = d.get("transformer_layers_per_block", 1)
    tl = tuple(tl) if isinstance(tl, (list, tuple)) else (tl,) * n
    down = tuple(d["down_block_types"])
    add = d.get("addition_embed_type") == "text_time"
    kw = dict(in_channels=d.get("in_channels", 4), out_channels=d.get("out_channels", 4), block_out_channels=chans,
              down_block_types=down, up_block_types=tuple(d["up_block_types"]),
              layers_per_block=d.get("layers_per_block", 2), transformer_layers_per_block=tl,
              cross_attention_dim=d.get("cross_attention_dim", 1280),
              use_linear_projection=bool(d.get("use_linear_projection", False)), addition_embed=add,
              norm_num_groups=d.get("norm_num_groups", 32), norm_eps=d.get("norm_eps", 1e-5))
    if len(widths) == 1:
        kw.update(head_dim=widths.pop(), num_heads=None)
    elif len(set(heads)) == 1:
        kw.update(head_dim=None, num_heads=heads[0])
    else:
        raise NotImplementedError(f"per-block head counts {heads} with differing head widths")
    if add:
        kw.update(addition_time_embed_dim=d.get("addition_time_embed_dim", 256),
                  projection_class_embeddings_input_dim=d.get("projection_class_embeddings_input_dim", 2816))
    return UNetConfig(**kw)


PAD_IN = 8    # conv_in input channels held (latent channels zero-padded)
PAD_OUT = 8   # conv_out output channels held


# ----------------------------------------------------------------------------------------------
# parameter specs in forward-execution order: (name, diffusers_shape, kind, fan_in)
def _lin(p, cin, cout, bias=True):
    out = [(p + ".weight", (cout, cin), "linear", cin)]
    if bias:
        out.append((p + ".bias", (cout,), "bias", cin))
    return out


def _conv(p, cin, cout, k=3):
    return [(p + ".weight", (cout, cin, k, k), "conv", cin * k * k), (p + ".bias", (cout,), "bias", cin * k * k)]


def _norm(p, c):
    return [(p + ".weight", (c,), "norm_w", 0), (p + ".bias", (c,), "norm_b", 0)]


def _resnet(p, cin, cout, cfg):
    s = _norm(p + ".norm1", cin) + _conv(p + ".conv1", cin, cout) + _lin(p + ".time_emb_proj", cfg.temb_dim, cout)
    s += _norm(p + ".norm2", cout) + _conv(p + ".conv2", cout, cout)
    if cin != cout:
        s += _conv(p + ".conv_shortcut", cin, cout, 1)
    return s


def _transformer(p, c, depth, cfg):
    s = _norm(p + ".norm", c)
    s += _lin(p + ".proj_in", c, c) if cfg.use_linear_projection else _conv(p + ".proj_in", c, c, 1)
    for k in range(depth):
        b = f"{p}.transformer_blocks.{k}"
        s += _norm(b + ".norm1", c)
        s += _lin(b + ".attn1.to_q", c, c, False) + _lin(b + ".attn1.to_k", c, c, False)
        s += _lin(b + ".attn1.to_v", c, c, False) + _lin(b + ".attn1.to_out.0", c, c)
        s += _norm(b + ".norm2", c)
        s += _lin(b + ".attn2.to_q", c, c, False)
        s += _lin(b + ".attn2.to_k", cfg.cross_attention_dim, c, False)
        s += _lin(b + ".attn2.to_v", cfg.cross_attention_dim, c, False)
        s += _lin(b + ".attn2.to_out.0", c, c)
        s += _norm(b + ".norm3", c)
        s += _lin(b + ".ff.net.0.proj", c, 8 * c) + _lin(b + ".ff.net.2", 4 * c, c)
    s += _lin(p + ".proj_out", c, c) if cfg.use_linear_projection else _conv(p + ".proj_out", c, c, 1)
    return s


def unet_specs(cfg: UNetConfig):
    ch = cfg.block_out_channels
    c0 = ch[0]
    s = _lin("time_embedding.linear_1", c0, cfg.temb_dim) + _lin("time_embedding.linear_2", cfg.temb_dim, cfg.temb_dim)
    if cfg.addition_embed:
        s += _lin("add_embedding.linear_1", cfg.projection_class_embeddings_input_dim, cfg.temb_dim)
        s += _lin("add_embedding.linear_2", cfg.temb_dim, cfg.temb_dim)
    s += _conv("conv_in", cfg.in_channels, c0)
    nlev = len(ch)
    skip = [c0]
    cin = c0
    for i, bt in enumerate(cfg.down_block_types):
        cout = ch[i]
        for j in range(cfg.layers_per_block):
            s += _resnet(f"down_blocks.{i}.resnets.{j}", cin if j == 0 else cout, cout, cfg)
            if bt.startswith("CrossAttn"):
                s += _transformer(f"down_blocks.{i}.attentions.{j}", cout, cfg.transformer_layers_per_block[i], cfg)
            skip.append(cout)
        if i < nlev - 1:
            s += _conv(f"down_blocks.{i}.downsamplers.0.conv", cout, cout)
            skip.append(cout)
        cin = cout
    s += _resnet("mid_block.resnets.0", ch[-1], ch[-1], cfg)
    s += _transformer("mid_block.attentions.0", ch[-1], cfg.transformer_layers_per_block[-1], cfg)
    s += _resnet("mid_block.resnets.1", ch[-1], ch[-1], cfg)
    rev = list(reversed(ch))
    rdepth = list(reversed(cfg.transformer_layers_per_block))
    prev = ch[-1]
    for i, bt in enumerate(cfg.up_block_types):
        cout = rev[i]
        for j in range(cfg.layers_per_block + 1):
            sk = skip.pop()
            s += _resnet(f"up_blocks.{i}.resnets.{j}", (prev if j == 0 else cout) + sk, cout, cfg)
            if bt.startswith("CrossAttn"):
                s += _transformer(f"up_blocks.{i}.attentions.{j}", cout, rdepth[i], cfg)
        if i < nlev - 1:
            s += _conv(f"up_blocks.{i}.upsamplers.0.conv", cout, cout)
        prev = cout
    s += _norm("conv_norm_out", c0) + _conv("conv_out", c0, cfg.out_channels)
    return s


def _store_shape(name, shape, kind, cfg):
    """internal layout: conv [Cout][kh][kw][Cin], 1x1 conv as linear, conv_in/out channel padding."""
    if kind == "conv":
        co, ci, kh, kw = shape
        if name == "conv_in.weight":
            ci = PAD_IN
        if name == "conv_out.weight":
            co = PAD_OUT
        if kh == 1:
            return (co, ci)
        return (co, kh, kw, ci)
    if name == "conv_out.bias":
        return (PAD_OUT,)
    return shape


class UNet2DConditionModel:
    """HIP UNet; parameters live in `self.store` (FlatParamStore)."""

    def __init__(self, cfg: UNetConfig, device, dtype=BF16, seed: int | None = 0, group: str = "unet",
                 trainable: bool = True, master: bool = False):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.specs = unet_specs(cfg)
        self.store = FlatParamStore([(n, _store_shape(n, sh, k, cfg), group) for n, sh, k, _ in self.specs],
                                    dtype, self.device, trainable=trainable, master=master)
        self._refs: dict = {}
        self.lora = None      # module/lora.py LoRAUNetWrapper when training adapters on a frozen base
        if seed is not None:
            self.init_weights(seed)

    # ----- parameters ---------------------------------------------------------------------------
    def init_weights(self, seed: int):
        """torch default init of diffusers modules: U(-1/sqrt(fan_in), 1/sqrt(fan_in)); norms 1/0."""
        g = torch.Generator(device=self.device).manual_seed(seed)
        with torch.no_grad():
            for name, shape, kind, fan_in in self.specs:
                p = self.store.params[name]
                if kind in ("linear", "conv", "bias"):
                    bound = 1.0 / math.sqrt(fan_in)
                    val = (torch.rand(shape, generator=g, device=self.device) * 2 - 1) * bound
                    self._assign(name, val, kind)
                elif kind == "norm_w":
                    self.store.write(name, torch.ones_like(p))
                else:
                    self.store.write(name, torch.zeros_like(p))

    def _assign(self, name, val_diffusers, kind):
        p = self.store.params[name]
        v = val_diffusers
        if kind == "conv":
            v = v.permute(0, 2, 3, 1) if v.dim() == 4 and v.shape[2] > 1 else v.reshape(v.shape[0], v.shape[1])
            if name == "conv_in.weight":
                v = torch.nn.functional.pad(v, (0, PAD_IN - v.shape[-1]))
            if name == "conv_out.weight":
                v = torch.nn.functional.pad(v, (0, 0, 0, 0, 0, 0, 0, PAD_OUT - v.shape[0]))
        if name == "conv_out.bias":
            v = torch.nn.functional.pad(v, (0, PAD_OUT - v.shape[0]))
        self.store.write(name, v)

    def named_parameters(self):
        return self.store.named_parameters()

    def parameters(self):
        return [p for _, p in self.store.named_parameters()]

    def num_parameters(self) -> int:
        return sum(math.prod(sh) for _, sh, _, _ in self.specs)

    def state_dict(self, dtype=None, grads=False):
        self.store.wait_params()
        """diffusers-layout state dict (NCHW conv weights, unpadded); grads=True exports gradients."""
        out = {}
        for name, shape, kind, _ in self.specs:
            v = self.store.params[name].grad if grads else self.store.value(name)
            if kind == "conv":
                if v.dim() == 2:
                    v = v.reshape(v.shape[0], v.shape[1], 1, 1)
                else:
                    v = v.permute(0, 3, 1, 2)
                v = v[:shape[0], :shape[1]]
            if name == "conv_out.bias":
                v = v[:shape[0]]
            out[name] = v.to(dtype or v.dtype).contiguous()
        return out

    def load_state_dict(self, sd):
        kinds = {n: k for n, _, k, _ in self.specs}
        with torch.no_grad():
            for name, shape, kind, _ in self.specs:
                if tuple(sd[name].shape) != tuple(shape):
                    raise ValueError(f"{name}: shape {tuple(sd[name].shape)} != {shape}")
                self._assign(name, sd[name].to(self.device, torch.float32), kinds[name])

    def R(self, names, shape=None) -> Fn.PRef:
        key = (tuple(names) if isinstance(names, (list, tuple)) else names, shape)
        r = self._refs.get(key)
        if r is None:
            r = Fn.PRef(self.store, names, shape)
            self._refs[key] = r
        return r

    # ----- blocks -------------------------------------------------------------------------------
    def _lo(self, module: str):
        """the LoRA site of a base module (None without adapters or when the filter excludes it)."""
        return self.lora.site_of.get(module) if self.lora is not None else None

    def _lo_fused(self, modules):
        """site of a fused base GEMM (to_q|to_k|to_v, to_k|to_v)."""
        return self.lora.site_for(list(modules)) if self.lora is not None else None

    def _linear(self, x, p, bias=True, residual=None):
        return Fn.linear(x, self.R(p + ".weight"), self.R(p + ".bias") if bias else None, residual, lora=self._lo(p))

    def _conv(self, x, p, rowvec=None, residual=None, stride=1, upsample=False):
        return Fn.conv(x, self.R(p + ".weight"), self.R(p + ".bias"), rowvec=rowvec, residual=residual, stride=stride,
                       upsample=upsample, lora=self._lo(p))

    def _gn(self, x, p, silu, eps=None):
        cfg = self.cfg
        return Fn.group_norm(x, self.R(p + ".weight"), self.R(p + ".bias"), cfg.norm_num_groups,
                             cfg.norm_eps if eps is None else eps, silu)

    def _gn_res(self, x, p, silu, eps=None):
        """(GroupNorm(x), alias of x for its residual / shortcut use): the two gradients of x meet in the
        GroupNorm backward (Fn.GroupNormResFn), not in an autograd add."""
        cfg = self.cfg
        return Fn.group_norm_res(x, self.R(p + ".weight"), self.R(p + ".bias"), cfg.norm_num_groups,
                                 cfg.norm_eps if eps is None else eps, silu)

    def _resnet(self, x, p, semb):
        h, x = self._gn_res(x, p + ".norm1", True)
        tp = self._linear(semb, p + ".time_emb_proj")
        h = self._conv(h, p + ".conv1", rowvec=tp)
        h = self._gn(h, p + ".norm2", True)
        sc = x
        if (p + ".conv_shortcut.weight") in self.store.slots:
            sc = self._linear(x, p + ".conv_shortcut")
        return self._conv(h, p + ".conv2", residual=sc)

    def _kv_batched(self, p, depth, C, ehs):
        """attn2.to_k|to_v of all `depth` blocks of one transformer as ONE batched GEMM over the text states
        (grid.y = block): each block's fused [2C, ctx] weight sits at the same stride in the flat store.
        The reference runs one [B*77, 2C] GEMM per block (70 per SDXL forward, ~25 us each at M = 308);
        this is 11 launches.  Backward stays per block (PrecomputedLinearFn).  None when not applicable
        (LoRA on the projection, a single block, irregular layout)."""
        if depth < 2 or self.lora is not None:
            return None
        names = [(f"{p}.transformer_blocks.{k}.attn2.to_k.weight", f"{p}.transformer_blocks.{k}.attn2.to_v.weight")
                 for k in range(depth)]
        offs = [self.store.slots[kn].offset for kn, _ in names]
        stride = offs[1] - offs[0]
        if any(offs[k + 1] - offs[k] != stride for k in range(depth - 1)) or stride % 8:
            return None
        ctxd = self.cfg.cross_attention_dim
        w0 = self.R(list(names[0]), (2 * C, ctxd)).w
        self.R(list(names[-1]), (2 * C, ctxd)).w   # orders after an in-flight optimizer update of the last block
        B_, L, _ = ehs.shape
        x = ehs.reshape(B_ * L, ctxd)
        if not x.is_contiguous():
            x = x.contiguous()
        out = torch.empty((depth, B_ * L, 2 * C), dtype=BF16, device=ehs.device)
        K.gemm_batched(x, ctxd, K.OPM_K, w0, ctxd, K.OPM_K, out, 2 * C, B_ * L, 2 * C, ctxd, depth, 1,
                       (0, 0), (stride, 0), (B_ * L * 2 * C, 0))
        return out.view(depth, B_, L, 2 * C)

    def _block(self, h, p, C, heads, ehs, kv_pre=None):
        B, N, _ = h.shape
        # norm1/2/3 hand back their input as the residual alias: its two gradients meet in one pass
        n1, h = Fn.layer_norm_res(h, self.R(p + ".norm1.weight"), self.R(p + ".norm1.bias"))
        wqkv = self.R([p + ".attn1.to_q.weight", p + ".attn1.to_k.weight", p + ".attn1.to_v.weight"], (3 * C, C))
        qkv = Fn.linear(n1, wqkv, lora=self._lo_fused([p + ".attn1.to_q", p + ".attn1.to_k", p + ".attn1.to_v"]))
        o = Fn.SelfAttnFn.apply(qkv, heads)
        h = self._linear(o, p + ".attn1.to_out.0", residual=h)
        n2, h = Fn.layer_norm_res(h, self.R(p + ".norm2.weight"), self.R(p + ".norm2.bias"))
        q = Fn.linear(n2, self.R(p + ".attn2.to_q.weight"), lora=self._lo(p + ".attn2.to_q"))
        ctxd = self.cfg.cross_attention_dim
        wkv = self.R([p + ".attn2.to_k.weight", p + ".attn2.to_v.weight"], (2 * C, ctxd))
        if kv_pre is not None:
            kv = Fn.precomputed_linear(ehs, wkv, kv_pre)
        else:
            kv = Fn.linear(ehs, wkv, lora=self._lo_fused([p + ".attn2.to_k", p + ".attn2.to_v"]))
        # dkv feeds only to_k|to_v's weight gradient (side stream) when the text states need no gradient: the batched
        # projection's (PrecomputedLinearFn) or the LoRA one's (LoraLinearFn runs its whole backward there then)
        o = Fn.CrossAttnFn.apply(q, kv, heads, (kv_pre is not None or (self.lora is not None and Fn._WONLY_SIDE))
                                 and not ehs.requires_grad)
        h = self._linear(o, p + ".attn2.to_out.0", residual=h)
        n3, h = Fn.layer_norm_res(h, self.R(p + ".norm3.weight"), self.R(p + ".norm3.bias"))
        g = self._linear(n3, p + ".ff.net.0.proj")
        a = Fn.GEGLUFn.apply(g)
        return self._linear(a, p + ".ff.net.2", residual=h)

    def _transformer(self, x, p, depth, ehs):
        B, H, W, C = x.shape
        heads = self.cfg.heads(C)
        h, x = self._gn_res(x, p + ".norm", False, eps=1e-6)
        h = self._linear(h.view(B, H * W, C), p + ".proj_in")
        kv_all = self._kv_batched(p, depth, C, ehs)
        for k in range(depth):
            h = self._block(h, f"{p}.transformer_blocks.{k}", C, heads, ehs, None if kv_all is None else kv_all[k])
        out = self._linear(h, p + ".proj_out", residual=x.view(B, H * W, C))
        return out.view(B, H, W, C)

    # ----- forward ------------------------------------------------------------------------------
    def __call__(self, sample, timestep, encoder_hidden_states, text_embeds=None, time_ids=None):
        return self.forward(sample, timestep, encoder_hidden_states, text_embeds, time_ids)

    def forward(self, sample, timestep, encoder_hidden_states, text_embeds=None, time_ids=None):
        """sample [B,H,W,8] bf16 NHWC (latent channels zero-padded), timestep int [B] or [1],
        encoder_hidden_states [B,L,ctx] bf16, SDXL: text_embeds [B,1280], time_ids [B,6].
        Returns the prediction [B,H,W,8] bf16 (channels >= out_channels are zero)."""
        cfg = self.cfg
        B = sample.shape[0]
        c0 = cfg.block_out_channels[0]
        t = timestep.reshape(-1)
        if t.numel() == 1 and B > 1:
            t = t.expand(B)
        t = t.to(torch.float32).contiguous()
        temb = self._linear(K.timestep_embedding(t, c0), "time_embedding.linear_1")
        temb = self._linear(Fn.SiLUFn.apply(temb), "time_embedding.linear_2")
        if cfg.addition_embed:
            te = K.timestep_embedding(time_ids.reshape(-1).to(torch.float32).contiguous(),
                                      cfg.addition_time_embed_dim).view(B, -1)
            add = torch.cat([text_embeds.to(BF16), te], dim=-1)
            a1 = self._linear(add, "add_embedding.linear_1")
            temb = self._linear(Fn.SiLUFn.apply(a1), "add_embedding.linear_2", residual=temb)
        semb = Fn.SiLUFn.apply(temb)
        ehs = encoder_hidden_states.to(BF16)

        x = self._conv(sample, "conv_in")
        skips = [x]
        nlev = len(cfg.block_out_channels)
        for i, bt in enumerate(cfg.down_block_types):
            for j in range(cfg.layers_per_block):
                x = self._resnet(x, f"down_blocks.{i}.resnets.{j}", semb)
                if bt.startswith("CrossAttn"):
                    x = self._transformer(x, f"down_blocks.{i}.attentions.{j}", cfg.transformer_layers_per_block[i], ehs)
                skips.append(x)
            if i < nlev - 1:
                x = self._conv(x, f"down_blocks.{i}.downsamplers.0.conv", stride=2)
                skips.append(x)
        x = self._resnet(x, "mid_block.resnets.0", semb)
        x = self._transformer(x, "mid_block.attentions.0", cfg.transformer_layers_per_block[-1], ehs)
        x = self._resnet(x, "mid_block.resnets.1", semb)
        rdepth = list(reversed(cfg.transformer_layers_per_block))
        for i, bt in enumerate(cfg.up_block_types):
            for j in range(cfg.layers_per_block + 1):
                x = Fn.ConcatFn.apply(x, skips.pop())
                x = self._resnet(x, f"up_blocks.{i}.resnets.{j}", semb)
                if bt.startswith("CrossAttn"):
                    x = self._transformer(x, f"up_blocks.{i}.attentions.{j}", rdepth[i], ehs)
            if i < nlev - 1:
                x = self._conv(x, f"up_blocks.{i}.upsamplers.0.conv", upsample=True)
        h = self._gn(x, "conv_norm_out", True)
        return self._conv(h, "conv_out")


def flops_per_image(cfg: UNetConfig, h: int, w: int, ctx_len: int = 77) -> float:
    """Analytic forward FLOPs per image (2 x MACs, norms/softmax excluded)."""
    macs = 0
    ch = cfg.block_out_channels
    c0 = ch[0]

    def res(hw, cin, cout):
        m = hw * cin * cout * 9 + hw * cout * cout * 9 + cfg.temb_dim * cout
        if cin != cout:
            m += hw * cin * cout
        return m

    def tr(hw, c, depth):
        m = 2 * hw * c * c
        for _ in range(depth):
            m += 4 * hw * c * c + 2 * hw * hw * c
            m += 2 * hw * c * c + 2 * ctx_len * cfg.cross_attention_dim * c + 2 * hw * ctx_len * c
            m += hw * c * 8 * c + hw * 4 * c * c
        return m

    hw = h * w
    macs += hw * cfg.in_channels * c0 * 9
    skip = [c0]
    cin = c0
    res_hw = hw
    nlev = len(ch)
    for i, bt in enumerate(cfg.down_block_types):
        cout = ch[i]
        for j in range(cfg.layers_per_block):
            macs += res(res_hw, cin if j == 0 else cout, cout)
            if bt.startswith("CrossAttn"):
                macs += tr(res_hw, cout, cfg.transformer_layers_per_block[i])
            skip.append(cout)
        if i < nlev - 1:
            macs += (res_hw // 4) * cout * cout * 9
            res_hw //= 4
            skip.append(cout)
        cin = cout
    macs += 2 * res(res_hw, ch[-1], ch[-1]) + tr(res_hw, ch[-1], cfg.transformer_layers_per_block[-1])
    rev = list(reversed(ch))
    rdepth = list(reversed(cfg.transformer_layers_per_block))
    prev = ch[-1]
    for i, bt in enumerate(cfg.up_block_types):
        cout = rev[i]
        for j in range(cfg.layers_per_block + 1):
            macs += res(res_hw, (prev if j == 0 else cout) + skip.pop(), cout)
            if bt.startswith("CrossAttn"):
                macs += tr(res_hw, cout, rdepth[i])
        if i < nlev - 1:
            res_hw *= 4
            macs += res_hw * cout * cout * 9
        prev = cout
    macs += hw * c0 * cfg.out_channels * 9
    return 2.0 * macs
