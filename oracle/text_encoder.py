"""CPU fp32 restatement of the text encoders the reference caches text states with, taking
transformers state-dict names.  TEST INFRASTRUCTURE ONLY (oracle/__init__.py).

  * CLIP text transformer (transformers CLIPTextModel / CLIPTextModelWithProjection): token +
    position embedding, pre-LN blocks (causal self-attention with biases, quick_gelu / erf-gelu MLP),
    final LayerNorm, pooled = final-normed state at argmax(ids), optional bias-free text projection;
  * T5 encoder (transformers T5EncoderModel, v1.1 gated-GELU FFN): RMS layer norm, unscaled
    attention scores + bucketed relative position bias from block 0, gelu_new(wi_0 x) * wi_1 x.
Selection of the cached tensors follows modules/model/util/clip_util.py:6-43 (encode_clip) and
modules/model/util/t5_util.py (encode_t5), called from StableDiffusionXLModel.py:233-256,
StableDiffusionModel.py:208-217 and FluxModel.py:235-262.

Pinning: transformers is importable here (the reference pins 4.48.3; the CLIP / T5 math is the
same in the installed 5.x) and tests/test_text_encoder.py checks this restatement against
transformers' own modules with random weights -- the reference's actual dependency.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _ln(x, w, b, eps):
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def _act(x, kind):
    if kind == "quick_gelu":
        return x * torch.sigmoid(1.702 * x)
    if kind == "gelu":
        return F.gelu(x)
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x ** 3)))


def clip_forward(sd: dict, ids: torch.Tensor, heads: int, act: str, eps: float = 1e-5):
    """-> (hidden_states list [emb, after layer 1, ..., after layer N] (un-normed), last_hidden_state,
    pooler_output, text_embeds or None)."""
    W = {k: v.float() for k, v in sd.items()}
    B, T = ids.shape
    x = W["text_model.embeddings.token_embedding.weight"][ids] + W["text_model.embeddings.position_embedding.weight"][:T]
    D = x.shape[-1]
    dh = D // heads
    mask = torch.full((T, T), float("-inf")).triu(1)
    hs = [x]
    i = 0
    while f"text_model.encoder.layers.{i}.layer_norm1.weight" in W:
        p = f"text_model.encoder.layers.{i}."
        h = _ln(x, W[p + "layer_norm1.weight"], W[p + "layer_norm1.bias"], eps)
        q, k, v = (h @ W[p + f"self_attn.{n}_proj.weight"].t() + W[p + f"self_attn.{n}_proj.bias"] for n in "qkv")
        q, k, v = (t.view(B, T, heads, dh).transpose(1, 2) for t in (q, k, v))
        a = torch.softmax(q @ k.transpose(-1, -2) * dh ** -0.5 + mask, dim=-1) @ v
        a = a.transpose(1, 2).reshape(B, T, D)
        x = x + a @ W[p + "self_attn.out_proj.weight"].t() + W[p + "self_attn.out_proj.bias"]
        h = _ln(x, W[p + "layer_norm2.weight"], W[p + "layer_norm2.bias"], eps)
        f = _act(h @ W[p + "mlp.fc1.weight"].t() + W[p + "mlp.fc1.bias"], act)
        x = x + f @ W[p + "mlp.fc2.weight"].t() + W[p + "mlp.fc2.bias"]
        hs.append(x)
        i += 1
    last = _ln(x, W["text_model.final_layer_norm.weight"], W["text_model.final_layer_norm.bias"], eps)
    pooled = last[torch.arange(B), ids.argmax(dim=-1)]
    embeds = pooled @ W["text_projection.weight"].t() if "text_projection.weight" in W else None
    return hs, last, pooled, embeds


def encode_clip(sd, ids, heads, act, default_layer=-1, layer_skip=0, add_layer_norm=True, eps=1e-5):
    hs, last, pooled, embeds = clip_forward(sd, ids, heads, act, eps)
    out = hs[default_layer - layer_skip]
    if add_layer_norm:
        out = _ln(out, sd["text_model.final_layer_norm.weight"].float(), sd["text_model.final_layer_norm.bias"].float(), eps)
    return out, (embeds if embeds is not None else pooled)


def t5_bucket(rel: torch.Tensor, num_buckets=32, max_distance=128) -> torch.Tensor:
    """T5Attention._relative_position_bucket, bidirectional."""
    nb = num_buckets // 2
    ret = (rel > 0).long() * nb
    n = rel.abs()
    max_exact = nb // 2
    large = max_exact + (torch.log(n.float() / max_exact) / math.log(max_distance / max_exact)
                         * (nb - max_exact)).long()
    large = torch.minimum(large, torch.full_like(large, nb - 1))
    return ret + torch.where(n < max_exact, n, large)


def t5_forward(sd: dict, ids: torch.Tensor, heads: int, eps: float = 1e-6, num_buckets=32, max_distance=128):
    """-> hidden_states list as transformers builds it: [emb, after block 0, ..., after block N-2,
    final_layer_norm(after block N-1)]."""
    W = {k: v.float() for k, v in sd.items()}
    B, T = ids.shape

    def rms(x, w):
        return w * (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps))

    x = W["shared.weight"][ids]
    pos = torch.arange(T)
    bucket = t5_bucket(pos[None, :] - pos[:, None], num_buckets, max_distance)
    bias = W["encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"][bucket].permute(2, 0, 1)
    hs = [x]
    i = 0
    while f"encoder.block.{i}.layer.0.layer_norm.weight" in W:
        p = f"encoder.block.{i}.layer."
        h = rms(x, W[p + "0.layer_norm.weight"])
        q, k, v = (h @ W[p + f"0.SelfAttention.{n}.weight"].t() for n in "qkv")
        dh = q.shape[-1] // heads
        q, k, v = (t.view(B, T, heads, dh).transpose(1, 2) for t in (q, k, v))
        a = torch.softmax(q @ k.transpose(-1, -2) + bias, dim=-1) @ v
        x = x + a.transpose(1, 2).reshape(B, T, -1) @ W[p + "0.SelfAttention.o.weight"].t()
        h = rms(x, W[p + "1.layer_norm.weight"])
        g = _act(h @ W[p + "1.DenseReluDense.wi_0.weight"].t(), "gelu_new") * (h @ W[p + "1.DenseReluDense.wi_1.weight"].t())
        x = x + g @ W[p + "1.DenseReluDense.wo.weight"].t()
        hs.append(x)
        i += 1
    hs[-1] = rms(x, W["encoder.final_layer_norm.weight"])
    return hs
