"""FLUX.1 transformer (FluxTransformer2DModel) on the HIP kernels, flat parameter store with diffusers
parameter names.  Drop-in for the network the reference calls at modules/modelSetup/BaseFluxSetup.py:289-299
(SURVEY.md §8(a) a10), with FluxModel.pack/unpack_latents (modules/model/FluxModel.py:300-344).

MI355X layout (not a translation of the diffusers module tree):
  * activations are rows r = t * B + b of the joint sequence [text (L) ; image (N)] -- a stream is a
    contiguous row block, so the double blocks' two streams, the single blocks and the joint
    attention share buffers and the reference's cat / split cost nothing;
  * every modulation Linear (norm1 / norm1_context / single norm / norm_out, ~3.2 B of FLUX.1-dev's
    weights) reads the same silu(temb): their weights are adjacent in the store and run as ONE
    [B, NMOD] GEMM that streams the weights once at HBM rate (per-module GEMMs only when a LoRA
    adapter sits on them);
  * q|k|v (and the add_*_proj triple) are one GEMM; in the single blocks q|k|v|proj_mlp share the
    input and run as ONE [T*B, 7D] GEMM whose attention / GELU halves feed proj_out in place.
"""
from __future__ import annotations

import contextlib
import math
import os
from dataclasses import dataclass

import numpy as np
import torch

from .. import kernels as K
from . import functional as Fn
from . import streams as S
from . import flux_ops as O
from .param_store import FlatParamStore

BF16 = torch.bfloat16


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



# the blocks' adaLN inputs are also their residuals: AdaLNResFn sums the two gradient contributions inside the adaLN
# backward (OTAMD_ADALN_RES=0: autograd adds them, the A/B reference)
_ADALN_RES = os.environ.get("OTAMD_ADALN_RES", "1") != "0"
# the embedders, the modulation GEMMs and the adaLN modulation sums on the weight-gradient stream (FluxTransformer.forward;
# OTAMD_MOD_SIDE=0: on the current stream, the A/B reference)
_MOD_SIDE = os.environ.get("OTAMD_MOD_SIDE", "1") != "0"


def _adaln_res(hx, emb, st, segs, B):
    if _ADALN_RES:
        return O.AdaLNResFn.apply(hx, emb, st, segs, B)
    return O.AdaLNFn.apply(hx, emb, st, segs, B), hx


def flux_dev_config() -> FluxConfig:
    return FluxConfig()


def tiny_flux_config() -> FluxConfig:
    return FluxConfig(num_layers=2, num_single_layers=2, num_attention_heads=2, joint_attention_dim=64,
                      pooled_projection_dim=32)


def _lin(p, cin, cout):
    return [(p + ".weight", (cout, cin), "linear", cin), (p + ".bias", (cout,), "bias", cin)]


def _fused(prefix, names, cin, cout):
    """weights of the modules adjacent, then their biases adjacent (one fused GEMM operand each)."""
    return [(f"{prefix}{n}.weight", (cout, cin), "linear", cin) for n in names] + \
        [(f"{prefix}{n}.bias", (cout,), "bias", cin) for n in names]


def modulation_modules(cfg: FluxConfig):
    """(module, n chunks) of every modulation Linear, in the fused GEMM's column order."""
    out = []
    for i in range(cfg.num_layers):
        out += [(f"transformer_blocks.{i}.norm1.linear", 6), (f"transformer_blocks.{i}.norm1_context.linear", 6)]
    out += [(f"single_transformer_blocks.{j}.norm.linear", 3) for j in range(cfg.num_single_layers)]
    out.append(("norm_out.linear", 2))
    return out


def flux_specs(cfg: FluxConfig):
    D = cfg.inner_dim
    hd = cfg.attention_head_dim
    s = []
    te = "time_text_embed."
    s += _lin(te + "timestep_embedder.linear_1", 256, D) + _lin(te + "timestep_embedder.linear_2", D, D)
    if cfg.guidance_embeds:
        s += _lin(te + "guidance_embedder.linear_1", 256, D) + _lin(te + "guidance_embedder.linear_2", D, D)
    s += _lin(te + "text_embedder.linear_1", cfg.pooled_projection_dim, D) + _lin(te + "text_embedder.linear_2", D, D)
    s += _lin("context_embedder", cfg.joint_attention_dim, D) + _lin("x_embedder", cfg.in_channels, D)
    mods = modulation_modules(cfg)
    s += [(m + ".weight", (n * D, D), "linear", D) for m, n in mods]
    s += [(m + ".bias", (n * D,), "bias", D) for m, n in mods]
    for i in range(cfg.num_layers):
        b = f"transformer_blocks.{i}."
        s += _fused(b + "attn.", ["to_q", "to_k", "to_v"], D, D)
        s += [(b + "attn.norm_q.weight", (hd,), "norm_w", 0), (b + "attn.norm_k.weight", (hd,), "norm_w", 0)]
        s += _fused(b + "attn.", ["add_q_proj", "add_k_proj", "add_v_proj"], D, D)
        s += [(b + "attn.norm_added_q.weight", (hd,), "norm_w", 0), (b + "attn.norm_added_k.weight", (hd,), "norm_w", 0)]
        s += _lin(b + "attn.to_out.0", D, D) + _lin(b + "attn.to_add_out", D, D)
        s += _lin(b + "ff.net.0.proj", D, 4 * D) + _lin(b + "ff.net.2", 4 * D, D)
        s += _lin(b + "ff_context.net.0.proj", D, 4 * D) + _lin(b + "ff_context.net.2", 4 * D, D)
    for j in range(cfg.num_single_layers):
        b = f"single_transformer_blocks.{j}."
        s += [(f"{b}attn.to_{x}.weight", (D, D), "linear", D) for x in "qkv"]
        s += [(b + "proj_mlp.weight", (4 * D, D), "linear", D)]
        s += [(f"{b}attn.to_{x}.bias", (D,), "bias", D) for x in "qkv"] + [(b + "proj_mlp.bias", (4 * D,), "bias", D)]
        s += [(b + "attn.norm_q.weight", (hd,), "norm_w", 0), (b + "attn.norm_k.weight", (hd,), "norm_w", 0)]
        s += _lin(b + "proj_out", 5 * D, D)
    s += _lin("proj_out", D, cfg.in_channels)
    return s


def flops_per_image(cfg: FluxConfig, n_img: int, n_txt: int = 77) -> float:
    """forward FLOPs per image (2 x MACs; 12 D^2 per token per block, 2 T^2 D
    attention per block, embedders; modulation / norms excluded)."""
    D, T = cfg.inner_dim, n_img + n_txt
    blocks = cfg.num_layers + cfg.num_single_layers
    macs = blocks * (T * 12 * D * D + 2 * T * T * D)
    macs += n_img * cfg.in_channels * D * 2 + n_txt * cfg.joint_attention_dim * D
    return 2.0 * macs


def rope_tables(L: int, h: int, w: int, cfg: FluxConfig):
    """cos / sin [L + (h/2)(w/2), 128] fp32 of FluxPosEmbed over cat(txt_ids = 0, img_ids) (float64 math,
    repeat-interleaved), as get_1d_rotary_pos_embed(use_real=True, repeat_interleave_real=True)."""
    ids = np.zeros((L + (h // 2) * (w // 2), 3), dtype=np.float64)
    yy, xx = np.meshgrid(np.arange(h // 2), np.arange(w // 2), indexing="ij")
    ids[L:, 1] = yy.reshape(-1)
    ids[L:, 2] = xx.reshape(-1)
    cos_l, sin_l = [], []
    for i, d in enumerate(cfg.axes_dims_rope):
        freqs = 1.0 / (cfg.theta ** (np.arange(0, d, 2, dtype=np.float64)[: d // 2] / d))
        f = np.outer(ids[:, i], freqs)
        cos_l.append(np.repeat(np.cos(f), 2, axis=1).astype(np.float32))
        sin_l.append(np.repeat(np.sin(f), 2, axis=1).astype(np.float32))
    return np.concatenate(cos_l, 1), np.concatenate(sin_l, 1)


class FluxTransformer2DModel:
    def __init__(self, cfg: FluxConfig, device, dtype=BF16, seed: int | None = 0, group: str = "transformer",
                 trainable: bool = True, master: bool = False):
        if cfg.attention_head_dim != 128 or sum(cfg.axes_dims_rope) != 128:
            raise NotImplementedError("the q/k norm + RoPE kernel is built for 128-wide heads")
        self.cfg = cfg
        self.device = torch.device(device)
        self.specs = flux_specs(cfg)
        self.store = FlatParamStore([(n, sh, group) for n, sh, _, _ in self.specs], dtype, self.device,
                                    trainable=trainable, master=master)
        self.config = {"guidance_embeds": cfg.guidance_embeds}
        self.lora = None
        self._refs: dict = {}
        self._rope: dict = {}
        self.mods = modulation_modules(cfg)
        D = cfg.inner_dim
        self.mod_off, off = {}, 0
        for m, n in self.mods:
            self.mod_off[m] = off
            off += n * D
        self.n_mod = off
        if seed is not None:
            self.init_weights(seed)

    # ----- parameters ---------------------------------------------------------------------------
    def init_weights(self, seed: int):
        """torch default init (U(+-1/sqrt(fan_in)) for Linear weight / bias), RMSNorm weights 1."""
        g = torch.Generator(device=self.device).manual_seed(seed)
        with torch.no_grad():
            for name, shape, kind, fan_in in self.specs:
                p = self.store.params[name]
                if kind in ("linear", "bias"):
                    b = 1.0 / math.sqrt(fan_in)
                    self.store.write(name, (torch.rand(shape, generator=g, device=self.device) * 2 - 1) * b)
                else:
                    self.store.write(name, torch.ones_like(p))

    def parameters(self):
        return [p for _, p in self.store.named_parameters()]

    def num_parameters(self) -> int:
        return sum(math.prod(sh) for _, sh, _, _ in self.specs)

    def state_dict(self, dtype=None, grads=False):
        self.store.wait_params()
        out = {}
        for name, *_ in self.specs:
            v = self.store.params[name].grad if grads else self.store.value(name)
            out[name] = v.to(dtype or v.dtype).contiguous()
        return out

    def load_state_dict(self, sd):
        with torch.no_grad():
            for name, shape, *_ in self.specs:
                if tuple(sd[name].shape) != tuple(shape):
                    raise ValueError(f"{name}: shape {tuple(sd[name].shape)} != {shape}")
                self.store.write(name, sd[name].to(self.device, torch.float32))

    def R(self, names, shape=None) -> Fn.PRef:
        key = (tuple(names) if isinstance(names, (list, tuple)) else names, shape)
        r = self._refs.get(key)
        if r is None:
            r = Fn.PRef(self.store, names, shape)
            self._refs[key] = r
        return r

    # ----- LoRA grouping (module/lora.py LoRAWrapper) -------------------------------------------
    def fused_group(self, name, by_name):
        base, _, leaf = name.rpartition(".")
        if name.endswith(".norm1.linear") or name.endswith(".norm1_context.linear"):
            blk = name.rsplit(".", 2)[0]
            return [blk + ".norm1.linear", blk + ".norm1_context.linear"]
        if name.startswith("transformer_blocks.") and leaf in ("to_q", "to_k", "to_v"):
            return [f"{base}.to_q", f"{base}.to_k", f"{base}.to_v"]
        if leaf in ("add_q_proj", "add_k_proj", "add_v_proj"):
            return [f"{base}.add_q_proj", f"{base}.add_k_proj", f"{base}.add_v_proj"]
        if name.startswith("single_transformer_blocks."):
            blk = name.split(".")[1]
            p = f"single_transformer_blocks.{blk}."
            if leaf in ("to_q", "to_k", "to_v") or name.endswith(".proj_mlp"):
                return [p + "attn.to_q", p + "attn.to_k", p + "attn.to_v", p + "proj_mlp"]
        return [name]

    def _site(self, modules):
        return self.lora.site_for(list(modules)) if self.lora is not None else None

    def _fused_lin(self, modules, cin):
        """(wref, bref, site) of a GEMM over adjacent modules."""
        n = sum(self.store.slots[m + ".weight"].shape[0] for m in modules)
        w = self.R([m + ".weight" for m in modules], (n, cin))
        b = self.R([m + ".bias" for m in modules], (n,))
        return w, b, self._site(modules)

    def _linear(self, x, m, residual=None):
        return Fn.linear(x, self.R(m + ".weight"), self.R(m + ".bias"), residual, lora=self._site([m]))

    def rope(self, L, h, w):
        key = (L, h, w)
        r = self._rope.get(key)
        if r is None:
            cs, sn = rope_tables(L, h, w, self.cfg)
            r = (torch.from_numpy(cs).to(self.device), torch.from_numpy(sn).to(self.device))
            self._rope[key] = r
        return r

    # ----- forward ------------------------------------------------------------------------------
    def _modulation(self, semb):
        """{module: (emb, state, column offset)} of every modulation Linear."""
        D = self.cfg.inner_dim
        adapted = self.lora is not None and any(self.lora.site_of.get(m) is not None for m, _ in self.mods)
        out = {}
        if not adapted:   # one GEMM over all modulation weights
            w = self.R([m + ".weight" for m, _ in self.mods], (self.n_mod, D))
            b = self.R([m + ".bias" for m, _ in self.mods], (self.n_mod,))
            emb = Fn.linear(semb, w, b)
            st = O.ModState(emb)
            for m, _ in self.mods:
                out[m] = (emb, st, self.mod_off[m])
            return out
        # LoRA on the modulation: one GEMM per block (both streams' norm1 of a double block fused)
        for i in range(self.cfg.num_layers):
            ms = [f"transformer_blocks.{i}.norm1.linear", f"transformer_blocks.{i}.norm1_context.linear"]
            w, b, site = self._fused_lin(ms, D)
            emb = Fn.linear(semb, w, b, lora=site)
            st = O.ModState(emb)
            out[ms[0]], out[ms[1]] = (emb, st, 0), (emb, st, 6 * D)
        for m, n in self.mods[2 * self.cfg.num_layers:]:
            emb = self._linear(semb, m)
            out[m] = (emb, O.ModState(emb), 0)
        return out

    def _embed_and_modulate(self, t_eff, g_eff, pooled_b):
        """time / guidance / pooled-text embedders -> silu(temb) -> every modulation GEMM (see _modulation)"""
        te = "time_text_embed."
        temb = self._linear(Fn.SiLUFn.apply(self._linear(K.timestep_embedding(t_eff, 256),
                                                         te + "timestep_embedder.linear_1")),
                            te + "timestep_embedder.linear_2")
        if g_eff is not None:
            temb = self._linear(Fn.SiLUFn.apply(self._linear(K.timestep_embedding(g_eff, 256),
                                                             te + "guidance_embedder.linear_1")),
                                te + "guidance_embedder.linear_2", residual=temb)
        temb = self._linear(Fn.SiLUFn.apply(self._linear(pooled_b, te + "text_embedder.linear_1")),
                            te + "text_embedder.linear_2", residual=temb)
        return self._modulation(Fn.SiLUFn.apply(temb))

    def forward(self, tokens, timestep, guidance, pooled, ehs, h, w):
        """tokens: packed image latents [N*B, in_channels] bf16, rows t*B + b (K.flux_pack);
        timestep: [B] fp32 = the reference's t / 1000; guidance [B] fp32 or None; pooled [B, P] bf16;
        ehs [B, L, joint_dim] bf16; h, w: latent size.  Returns the predicted packed flow [N*B, in_channels]."""
        cfg = self.cfg
        D, H = cfg.inner_dim, cfg.num_attention_heads
        B, L, _ = ehs.shape
        N = (h // 2) * (w // 2)
        T = L + N
        # diffusers: timestep.to(bf16) * 1000 in bf16, then the fp32 sinusoid (BaseFluxSetup passes t / 1000)
        t_eff = (timestep.to(BF16) * 1000).float().contiguous()
        g_eff = (guidance.to(BF16) * 1000).float().contiguous() if cfg.guidance_embeds else None
        pooled_b = pooled.to(BF16).contiguous()
        # The embedders and every modulation GEMM run on the weight-gradient stream: their autograd nodes then run their
        # backward there too (torch runs a node's backward on its forward stream and orders the streams at each edge)
        # -- that branch only feeds weight gradients -- and the adaLN modulation sums follow (flux_ops._dmod_side).
        # (Not while a step graph is captured.)
        side = S.side_stream() if _MOD_SIDE and not torch.cuda.is_current_stream_capturing() else None
        if side is not None:
            side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            mod = self._embed_and_modulate(t_eff, g_eff, pooled_b)
        if side is not None:
            for u in (t_eff, g_eff, pooled_b):
                if u is not None:
                    u.record_stream(side)
            S.join()   # the blocks read the modulation vectors
            main = torch.cuda.current_stream()
            for emb, st, _ in {id(v[1]): v for v in mod.values()}.values():
                emb.record_stream(main)
                st.d.record_stream(main)
                st.side = True

        ctx_in = ehs.to(BF16).transpose(0, 1).reshape(L * B, -1)        # rows t*B + b
        hx = torch.cat([self._linear(ctx_in, "context_embedder"), self._linear(tokens, "x_embedder")], 0)
        rope = self.rope(L, h, w)
        LB, TB = L * B, T * B
        geo = (T, B, H, L)

        for i in range(cfg.num_layers):
            p = f"transformer_blocks.{i}."
            emb, st, o = mod[p + "norm1.linear"]
            embc, stc, oc = mod[p + "norm1_context.linear"]
            n, hx = _adaln_res(hx, emb, st, [(0, LB, oc, oc + D), (LB, TB, o, o + D)], B)
            wi, bi, si = self._fused_lin([p + "attn.to_q", p + "attn.to_k", p + "attn.to_v"], D)
            wc, bc, sc = self._fused_lin([p + "attn.add_q_proj", p + "attn.add_k_proj", p + "attn.add_v_proj"], D)
            qkv = O.rows_linear(n, [(0, LB, wc, bc, sc), (LB, TB, wi, bi, si)])
            norms = (self.R(p + "attn.norm_q.weight"), self.R(p + "attn.norm_k.weight"),
                     self.R(p + "attn.norm_added_q.weight"), self.R(p + "attn.norm_added_k.weight"))
            a = O.JointAttnFn.apply(qkv, geo, norms, rope, *Fn._trainable_params(*norms))
            ao = O.rows_linear(a, [(0, LB, self.R(p + "attn.to_add_out.weight"), self.R(p + "attn.to_add_out.bias"),
                                    self._site([p + "attn.to_add_out"])),
                                   (LB, TB, self.R(p + "attn.to_out.0.weight"), self.R(p + "attn.to_out.0.bias"),
                                    self._site([p + "attn.to_out.0"]))])
            hx = O.GatedAddFn.apply(hx, ao, emb, st, [(0, LB, oc + 2 * D), (LB, TB, o + 2 * D)], B)
            n2, hx = _adaln_res(hx, emb, st, [(0, LB, oc + 3 * D, oc + 4 * D), (LB, TB, o + 3 * D, o + 4 * D)],
                                        B)
            f1 = O.rows_linear(n2, [(0, LB, self.R(p + "ff_context.net.0.proj.weight"),
                                     self.R(p + "ff_context.net.0.proj.bias"), self._site([p + "ff_context.net.0.proj"])),
                                    (LB, TB, self.R(p + "ff.net.0.proj.weight"), self.R(p + "ff.net.0.proj.bias"),
                                     self._site([p + "ff.net.0.proj"]))])
            gl = O.GeluTanhFn.apply(f1)
            f2 = O.rows_linear(gl, [(0, LB, self.R(p + "ff_context.net.2.weight"), self.R(p + "ff_context.net.2.bias"),
                                     self._site([p + "ff_context.net.2"])),
                                    (LB, TB, self.R(p + "ff.net.2.weight"), self.R(p + "ff.net.2.bias"),
                                     self._site([p + "ff.net.2"]))])
            hx = O.GatedAddFn.apply(hx, f2, emb, st, [(0, LB, oc + 5 * D), (LB, TB, o + 5 * D)], B)

        geo1 = (T, B, H, 0)
        for j in range(cfg.num_single_layers):
            p = f"single_transformer_blocks.{j}."
            emb, st, o = mod[p + "norm.linear"]
            n, hx = _adaln_res(hx, emb, st, [(0, TB, o, o + D)], B)
            wu, bu, su = self._fused_lin([p + "attn.to_q", p + "attn.to_k", p + "attn.to_v", p + "proj_mlp"], D)
            u = Fn.linear(n, wu, bu, lora=su)
            norms = (self.R(p + "attn.norm_q.weight"), self.R(p + "attn.norm_k.weight"), None, None)
            cat = O.SingleMixFn.apply(u, geo1, norms, rope, *Fn._trainable_params(*norms[:2]))
            po = self._linear(cat, p + "proj_out")
            hx = O.GatedAddFn.apply(hx, po, emb, st, [(0, TB, o + 2 * D)], B)

        emb, st, o = mod["norm_out.linear"]
        img = hx[LB:]
        n = O.AdaLNFn.apply(img, emb, st, [(0, N * B, o + D, o)], B)   # AdaLayerNormContinuous: (scale, shift)
        return self._linear(n, "proj_out")

    __call__ = forward


def rows_per_image(module: str, L: int, N: int) -> int:
    """token rows one image contributes to a module's GEMM (text stream L, image stream N, both L + N,
    modulation / time embedders 1)."""
    if module.startswith("time_text_embed.") or module.endswith(".norm1.linear") or \
            module.endswith(".norm1_context.linear") or module.endswith(".norm.linear") or module == "norm_out.linear":
        return 1
    if module.startswith("single_transformer_blocks."):
        return L + N
    if module == "context_embedder" or ".add_" in module or ".to_add_out" in module or ".ff_context." in module:
        return L
    return N


def lora_macs_per_image(wrapper, L: int, N: int) -> float:
    """algorithmic forward MACs of the LoRA branches: rows x r x (cin + cout) per adapted module."""
    macs = 0.0
    for s in wrapper.sites:
        for m, co in zip(s.modules, s.couts_ref):
            macs += rows_per_image(m, L, N) * wrapper.rank * (s.cin_ref + co)
    return macs
