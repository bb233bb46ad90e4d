"""Frozen text encoders for text-state caching on the MI355X kernels.

  * CLIPTextEncoder: transformers' CLIPTextModel / CLIPTextModelWithProjection forward (SD 1.5
    text_encoder = CLIP-L, SDXL text_encoder = CLIP-L and text_encoder_2 = OpenCLIP bigG with its
    text projection; FLUX.1 text_encoder = CLIP-L for the pooled vector);
  * T5TextEncoder: transformers' T5EncoderModel forward (FLUX.1 text_encoder_2, T5 v1.1 XXL).
Both take token ids (tokenization is host-side text processing: the CLIP BPE / sentencepiece vocab
files ship with the checkpoints, which are not on this box) and return the tensors the reference
caches, selected exactly like modules/model/util/clip_util.py:6-43 (encode_clip) and
modules/model/util/t5_util.py (encode_t5):
  hidden_states[default_layer - layer_skip] (+ the final layer norm when add_layer_norm), and the
  pooled output (text_embeds with a projection, else pooler_output = final-normed state at the
  first highest token id, i.e. the EOS token).
Parameter names are the transformers state-dict names, so `load_state_dict` takes a checkpoint's
`text_encoder/` weights as they are.  Compute: bf16 MFMA GEMMs with fused bias / residual
epilogues, LayerNorm / RMSNorm kernels, materialized attention with the causal mask (CLIP) or the
relative position bias (T5) folded into the row softmax (csrc/text.hip).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from .. import kernels as K
from .param_store import FlatParamStore

BF16 = torch.bfloat16


@dataclass
class CLIPTextConfig:
    vocab_size: int = 49408
    hidden_size: int = 768
    intermediate_size: int = 3072
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    max_position_embeddings: int = 77
    hidden_act: str = "quick_gelu"
    layer_norm_eps: float = 1e-5
    projection_dim: int | None = None     # CLIPTextModelWithProjection (bigG: 1280, no bias)


def clip_l_config() -> CLIPTextConfig:
    return CLIPTextConfig()


def clip_bigg_config() -> CLIPTextConfig:
    return CLIPTextConfig(hidden_size=1280, intermediate_size=5120, num_hidden_layers=32, num_attention_heads=20,
                          hidden_act="gelu", projection_dim=1280)


def tiny_clip_config(projection: bool = False) -> CLIPTextConfig:
    return CLIPTextConfig(vocab_size=1000, hidden_size=64, intermediate_size=128, num_hidden_layers=3,
                          num_attention_heads=2, hidden_act="gelu" if projection else "quick_gelu",
                          projection_dim=64 if projection else None)


@dataclass
class T5Config:
    vocab_size: int = 32128
    d_model: int = 4096
    d_kv: int = 64
    d_ff: int = 10240
    num_layers: int = 24
    num_heads: int = 64
    relative_attention_num_buckets: int = 32
    relative_attention_max_distance: int = 128
    layer_norm_epsilon: float = 1e-6


def t5_xxl_config() -> T5Config:
    return T5Config()


def tiny_t5_config() -> T5Config:
    return T5Config(vocab_size=1000, d_model=64, d_kv=8, d_ff=96, num_layers=3, num_heads=8)


_ACT = {"quick_gelu": K.ACT_QUICK_GELU, "gelu": K.ACT_GELU_ERF, "gelu_new": K.ACT_GELU_TANH}


def clip_specs(c: CLIPTextConfig):
    D, F = c.hidden_size, c.intermediate_size
    s = [("text_model.embeddings.token_embedding.weight", (c.vocab_size, D)),
         ("text_model.embeddings.position_embedding.weight", (c.max_position_embeddings, D))]
    for i in range(c.num_hidden_layers):
        p = f"text_model.encoder.layers.{i}."
        s += [(p + "layer_norm1.weight", (D,)), (p + "layer_norm1.bias", (D,))]
        s += [(p + f"self_attn.{n}_proj.weight", (D, D)) for n in "qkv"]      # adjacent: one fused GEMM
        s += [(p + f"self_attn.{n}_proj.bias", (D,)) for n in "qkv"]
        s += [(p + "self_attn.out_proj.weight", (D, D)), (p + "self_attn.out_proj.bias", (D,)),
              (p + "layer_norm2.weight", (D,)), (p + "layer_norm2.bias", (D,)),
              (p + "mlp.fc1.weight", (F, D)), (p + "mlp.fc1.bias", (F,)),
              (p + "mlp.fc2.weight", (D, F)), (p + "mlp.fc2.bias", (D,))]
    s += [("text_model.final_layer_norm.weight", (D,)), ("text_model.final_layer_norm.bias", (D,))]
    if c.projection_dim:
        s += [("text_projection.weight", (c.projection_dim, D))]
    return s


def t5_specs(c: T5Config):
    D, I = c.d_model, c.num_heads * c.d_kv
    s = [("shared.weight", (c.vocab_size, D))]
    for i in range(c.num_layers):
        p = f"encoder.block.{i}.layer."
        s += [(p + "0.layer_norm.weight", (D,))]
        s += [(p + f"0.SelfAttention.{n}.weight", (I, D)) for n in "qkv"]
        s += [(p + "0.SelfAttention.o.weight", (D, I))]
        if i == 0:
            s += [(p + "0.SelfAttention.relative_attention_bias.weight", (c.relative_attention_num_buckets, c.num_heads))]
        s += [(p + "1.layer_norm.weight", (D,)), (p + "1.DenseReluDense.wi_0.weight", (c.d_ff, D)),
              (p + "1.DenseReluDense.wi_1.weight", (c.d_ff, D)), (p + "1.DenseReluDense.wo.weight", (D, c.d_ff))]
    s += [("encoder.final_layer_norm.weight", (D,))]
    return s


class _Frozen:
    def __init__(self, specs, device, seed):
        self.specs = specs
        self.device = device
        self.store = FlatParamStore([(n, sh, "text") for n, sh in specs], BF16, device, trainable=False)
        g = torch.Generator(device="cpu").manual_seed(seed)
        with torch.no_grad():
            for n, sh in specs:
                p = self.store.params[n]
                if "layer_norm" in n and n.endswith(".weight"):
                    p.fill_(1.0)
                elif n.endswith(".bias"):
                    p.zero_()
                else:
                    p.copy_((torch.randn(sh, generator=g) * 0.02).to(BF16))

    def W(self, name) -> torch.Tensor:
        return self.store.params[name].data

    def Wcat(self, names) -> torch.Tensor:
        return self.store.view(names)

    def state_dict(self, dtype=None) -> dict:
        return {n: self.store.params[n].detach().to(dtype or BF16).clone() for n, _ in self.specs}

    def load_state_dict(self, sd: dict) -> None:
        with torch.no_grad():
            for n, sh in self.specs:
                if n not in sd:
                    raise KeyError(f"missing text-encoder parameter {n}")
                if tuple(sd[n].shape) != tuple(sh):
                    raise ValueError(f"{n}: shape {tuple(sd[n].shape)} != {sh}")
                self.store.params[n].copy_(sd[n].to(self.device, BF16))


class CLIPTextEncoder(_Frozen):
    def __init__(self, cfg: CLIPTextConfig, device, seed=0):
        super().__init__(clip_specs(cfg), device, seed)
        self.cfg = cfg

    def forward(self, ids: torch.Tensor, want_layers: set[int] | None = None):
        """ids int64 [B, T] -> (hidden_states dict {index: [B, T, D]} for the requested indices of
        the transformers hidden_states tuple (0 = embeddings, i = after layer i), final-normed last
        state [B*T, D])."""
        c = self.cfg
        B, T = ids.shape
        D, H = c.hidden_size, c.num_attention_heads
        N = c.num_hidden_layers
        want = {(i % (N + 1)) for i in (want_layers or set())}
        x = K.embed_tokens(ids.contiguous(), self.W("text_model.embeddings.token_embedding.weight"),
                           self.W("text_model.embeddings.position_embedding.weight"))
        hs = {}
        if 0 in want:
            hs[0] = x.view(B, T, D)
        act = _ACT[c.hidden_act]
        scale = (D // H) ** -0.5
        for i in range(N):
            p = f"text_model.encoder.layers.{i}."
            h, _ = K.layernorm_fwd(x, self.W(p + "layer_norm1.weight"), self.W(p + "layer_norm1.bias"), c.layer_norm_eps)
            qkv = K.linear(h, self.Wcat([p + f"self_attn.{n}_proj.weight" for n in "qkv"]).view(3 * D, D),
                           bias=self.Wcat([p + f"self_attn.{n}_proj.bias" for n in "qkv"]).view(3 * D))
            q3 = qkv.view(B, T, 3 * D)
            o = K.attn_masked_fwd(q3[:, :, :D], q3[:, :, D:2 * D], q3[:, :, 2 * D:], H, scale=scale, causal=True)
            x = K.linear(o.view(B * T, D), self.W(p + "self_attn.out_proj.weight"),
                         bias=self.W(p + "self_attn.out_proj.bias"), residual=x)
            h, _ = K.layernorm_fwd(x, self.W(p + "layer_norm2.weight"), self.W(p + "layer_norm2.bias"), c.layer_norm_eps)
            f = K.act_fwd(K.linear(h, self.W(p + "mlp.fc1.weight"), bias=self.W(p + "mlp.fc1.bias")), act)
            x = K.linear(f, self.W(p + "mlp.fc2.weight"), bias=self.W(p + "mlp.fc2.bias"), residual=x)
            if i + 1 in want:
                hs[i + 1] = x.view(B, T, D)
        last, _ = K.layernorm_fwd(x, self.W("text_model.final_layer_norm.weight"),
                                  self.W("text_model.final_layer_norm.bias"), c.layer_norm_eps)
        return hs, last

    def pooled(self, ids: torch.Tensor, last: torch.Tensor) -> torch.Tensor:
        """pooler_output (final-normed state at argmax(ids), the EOS token of CLIP's vocab), projected
        by text_projection when the model has one (text_embeds)."""
        B, T = ids.shape
        eos = ids.argmax(dim=-1)                              # index glue (B values)
        rows = last.view(B, T, -1)[torch.arange(B, device=ids.device), eos].contiguous()
        if self.cfg.projection_dim:
            return K.linear(rows, self.W("text_projection.weight"))
        return rows

    def encode(self, ids, default_layer=-1, layer_skip=0, add_output=True, add_pooled_output=False,
               add_layer_norm=True):
        """encode_clip (clip_util.py:6-43) for one encoder: (hidden_states[default_layer - layer_skip]
        [B, T, D], final-normed when add_layer_norm; pooled) -- None where not requested."""
        N = self.cfg.num_hidden_layers
        idx = (default_layer - layer_skip) % (N + 1)
        hs, last = self.forward(ids, {idx} if add_output else set())
        out = None
        if add_output:
            if add_layer_norm and idx == N:
                out = last.view(*ids.shape, -1)           # last_hidden_state
            elif add_layer_norm:
                B, T, D = hs[idx].shape
                out, _ = K.layernorm_fwd(hs[idx].reshape(B * T, D), self.W("text_model.final_layer_norm.weight"),
                                         self.W("text_model.final_layer_norm.bias"), self.cfg.layer_norm_eps)
                out = out.view(B, T, D)
            else:
                out = hs[idx]
        pooled = self.pooled(ids, last) if add_pooled_output else None
        return out, pooled


def t5_relative_buckets(T: int, num_buckets: int, max_distance: int) -> np.ndarray:
    """T5Attention._relative_position_bucket, bidirectional (encoder): int64 [T, T] (query, key)."""
    ctx = np.arange(T, dtype=np.int64)[:, None]
    mem = np.arange(T, dtype=np.int64)[None, :]
    rel = mem - ctx
    nb = num_buckets // 2
    ret = (rel > 0).astype(np.int64) * nb
    n = np.abs(rel)
    max_exact = nb // 2
    is_small = n < max_exact
    nf = np.maximum(n, 1).astype(np.float32)          # n < max_exact takes the exact branch below
    large = max_exact + (np.log(nf / max_exact) / math.log(max_distance / max_exact) * (nb - max_exact)).astype(np.int64)
    large = np.minimum(large, nb - 1)
    return ret + np.where(is_small, n, large)


class T5TextEncoder(_Frozen):
    def __init__(self, cfg: T5Config, device, seed=0):
        super().__init__(t5_specs(cfg), device, seed)
        self.cfg = cfg
        self._bias_cache = {}

    def _position_bias(self, T: int) -> torch.Tensor:
        """[T*T, H] bf16: relative_attention_bias[bucket(q, c)] gathered by the embedding kernel."""
        b = self._bias_cache.get(T)
        if b is None:
            c = self.cfg
            ids = torch.from_numpy(t5_relative_buckets(T, c.relative_attention_num_buckets,
                                                       c.relative_attention_max_distance)).reshape(1, T * T)
            table = self.W("encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight")
            H = c.num_heads
            if H % 8:
                raise ValueError("T5 head count must be a multiple of 8 for the bias gather")
            b = K.embed_tokens(ids.to(self.device), table.contiguous())
            self._bias_cache[T] = b
        return b

    def forward(self, ids: torch.Tensor, want_layers: set[int] | None = None):
        """-> (hidden_states dict {index: [B, T, D]} (index N = after the final layer norm, as in
        transformers' tuple), final-normed last state [B*T, D])."""
        c = self.cfg
        B, T = ids.shape
        D, H, dk = c.d_model, c.num_heads, c.d_kv
        I = H * dk
        N = c.num_layers
        want = {(i % (N + 1)) for i in (want_layers or set())}
        x = K.embed_tokens(ids.contiguous(), self.W("shared.weight"))
        hs = {}
        if 0 in want:
            hs[0] = x.view(B, T, D)
        bias = self._position_bias(T)
        for i in range(N):
            p = f"encoder.block.{i}.layer."
            h = K.rmsnorm_fwd(x, self.W(p + "0.layer_norm.weight"), c.layer_norm_epsilon)
            qkv = K.linear(h, self.Wcat([p + f"0.SelfAttention.{n}.weight" for n in "qkv"]).view(3 * I, D))
            q3 = qkv.view(B, T, 3 * I)
            # scores unscaled (T5 folds 1/sqrt(d) into the init); bias[q, c, h] at (q*T + c)*H + h
            o = K.attn_masked_fwd(q3[:, :, :I], q3[:, :, I:2 * I], q3[:, :, 2 * I:], H, scale=1.0, bias=bias,
                                  bias_strides=(T * H, H, 1))
            x = K.linear(o.view(B * T, I), self.W(p + "0.SelfAttention.o.weight"), residual=x)
            h = K.rmsnorm_fwd(x, self.W(p + "1.layer_norm.weight"), c.layer_norm_epsilon)
            g = K.linear(h, self.Wcat([p + "1.DenseReluDense.wi_0.weight", p + "1.DenseReluDense.wi_1.weight"])
                         .view(2 * c.d_ff, D))
            f = K.gated_act_fwd(g, K.ACT_GELU_TANH)
            x = K.linear(f, self.W(p + "1.DenseReluDense.wo.weight"), residual=x)
            if i + 1 in want and i + 1 < N:
                hs[i + 1] = x.view(B, T, D)
        last = K.rmsnorm_fwd(x, self.W("encoder.final_layer_norm.weight"), c.layer_norm_epsilon)
        if N in want:
            hs[N] = last.view(B, T, D)
        return hs, last

    def encode(self, ids, default_layer=-1, layer_skip=0, add_layer_norm=True):
        """encode_t5 (t5_util.py): hidden_states[default_layer - layer_skip], final-normed when that
        is not already the last entry and add_layer_norm."""
        N = self.cfg.num_layers
        idx = (default_layer - layer_skip) % (N + 1)
        hs, _ = self.forward(ids, {idx})
        out = hs[idx]
        if idx != N and add_layer_norm:
            B, T, D = out.shape
            out = K.rmsnorm_fwd(out.reshape(B * T, D).contiguous(), self.W("encoder.final_layer_norm.weight"),
                                self.cfg.layer_norm_epsilon).view(B, T, D)
        return out


# ---- per-family text-state caching (the tensors the data loader caches and the step reads) ------
def encode_sdxl_text(te1: CLIPTextEncoder, te2: CLIPTextEncoder, tokens_1, tokens_2, layer_skip_1=0, layer_skip_2=0):
    """StableDiffusionXLModel.encode_text (:199-286): penultimate CLIP-L and bigG states without the
    final norm, bigG text_embeds as the pooled vector (dropout p = 0: the training default)."""
    h1, _ = te1.encode(tokens_1, default_layer=-2, layer_skip=layer_skip_1, add_layer_norm=False)
    h2, pooled = te2.encode(tokens_2, default_layer=-2, layer_skip=layer_skip_2, add_pooled_output=True,
                            add_layer_norm=False)
    return {"text_encoder_1_hidden_state": h1, "text_encoder_2_hidden_state": h2,
            "text_encoder_2_pooled_state": pooled}


def encode_sd15_text(te: CLIPTextEncoder, tokens, layer_skip=0):
    """StableDiffusionModel.encode_text (:208-217): last CLIP-L state (clip skip aware) + final norm."""
    h, _ = te.encode(tokens, default_layer=-1, layer_skip=layer_skip, add_layer_norm=True)
    return {"text_encoder_hidden_state": h}


def encode_flux_text(te1: CLIPTextEncoder, te2: T5TextEncoder, tokens_1, tokens_2, layer_skip_2=0):
    """FluxModel.encode_text (:235-262): CLIP-L pooler_output + T5 last hidden state."""
    _, pooled = te1.encode(tokens_1, add_output=False, add_pooled_output=True)
    h2 = te2.encode(tokens_2, default_layer=-1, layer_skip=layer_skip_2)
    return {"text_encoder_1_pooled_state": pooled, "text_encoder_2_hidden_state": h2}
