"""diffusers <-> original (LDM / "ckpt") parameter names for the UNet and the VAE encoder.

The reference converts diffusers state dicts to the single-file layout with explicit tables
(modules/util/convert/convert_sdxl_diffusers_to_ckpt.py:8-81 for SDXL, convert_sd_diffusers_to_ckpt.py
for SD 1.5, the shared pieces in convert_diffusers_to_ckpt_util.py:232-291); it reads single files
back through diffusers' from_single_file.  Here the same correspondence is derived from the block
structure of the build's own spec list, so one function serves SDXL and SD 1.5 in both directions:

  conv_in                       -> input_blocks.0.0
  time_embedding.linear_{1,2}   -> time_embed.{0,2}
  add_embedding.linear_{1,2}    -> label_emb.0.{0,2}
  down_blocks.i.resnets.j       -> input_blocks.(1 + i(L+1) + j).0      (L = layers_per_block)
  down_blocks.i.attentions.j    -> input_blocks.(1 + i(L+1) + j).1
  down_blocks.i.downsamplers.0  -> input_blocks.(1 + i(L+1) + L).0.op
  mid_block.{resnets.0, attentions.0, resnets.1} -> middle_block.{0, 1, 2}
  up_blocks.i.resnets.j         -> output_blocks.(i(L+1) + j).0
  up_blocks.i.attentions.j      -> output_blocks.(i(L+1) + j).1
  up_blocks.i.upsamplers.0      -> output_blocks.(i(L+1) + L).(2 if the block has attentions else 1)
  conv_norm_out / conv_out      -> out.0 / out.2
  resnet norm1 conv1 time_emb_proj norm2 conv2 conv_shortcut
                                -> in_layers.0 in_layers.2 emb_layers.1 out_layers.0 out_layers.3 skip_connection
Transformer2D internals keep their names.  Single files carry the prefixes
`model.diffusion_model.` (UNet) and `first_stage_model.` (VAE).
"""
from __future__ import annotations

import re

UNET_PREFIX = "model.diffusion_model."
VAE_PREFIX = "first_stage_model."

_RESNET = {"norm1": "in_layers.0", "conv1": "in_layers.2", "time_emb_proj": "emb_layers.1", "norm2": "out_layers.0",
           "conv2": "out_layers.3", "conv_shortcut": "skip_connection"}


def _resnet(rest: str) -> str:
    head, _, leaf = rest.partition(".")
    return f"{_RESNET[head]}.{leaf}"


def unet_ldm_name(name: str, cfg) -> str:
    L = cfg.layers_per_block
    up_attn = [t.startswith("CrossAttn") for t in cfg.up_block_types]
    fixed = {"conv_in": "input_blocks.0.0", "time_embedding.linear_1": "time_embed.0",
             "time_embedding.linear_2": "time_embed.2", "add_embedding.linear_1": "label_emb.0.0",
             "add_embedding.linear_2": "label_emb.0.2", "conv_norm_out": "out.0", "conv_out": "out.2"}
    mod, _, leaf = name.rpartition(".")
    if mod in fixed:
        return f"{fixed[mod]}.{leaf}"
    m = re.match(r"down_blocks\.(\d+)\.(resnets|attentions|downsamplers)\.(\d+)\.(.*)$", name)
    if m:
        i, kind, j, rest = int(m[1]), m[2], int(m[3]), m[4]
        if kind == "downsamplers":
            return f"input_blocks.{1 + i * (L + 1) + L}.0.op.{rest.removeprefix('conv.')}"
        idx = 1 + i * (L + 1) + j
        return f"input_blocks.{idx}.0.{_resnet(rest)}" if kind == "resnets" else f"input_blocks.{idx}.1.{rest}"
    m = re.match(r"mid_block\.(resnets|attentions)\.(\d+)\.(.*)$", name)
    if m:
        kind, j, rest = m[1], int(m[2]), m[3]
        if kind == "attentions":
            return f"middle_block.1.{rest}"
        return f"middle_block.{0 if j == 0 else 2}.{_resnet(rest)}"
    m = re.match(r"up_blocks\.(\d+)\.(resnets|attentions|upsamplers)\.(\d+)\.(.*)$", name)
    if m:
        i, kind, j, rest = int(m[1]), m[2], int(m[3]), m[4]
        if kind == "upsamplers":
            return f"output_blocks.{i * (L + 1) + L}.{2 if up_attn[i] else 1}.{rest}"
        idx = i * (L + 1) + j
        return f"output_blocks.{idx}.0.{_resnet(rest)}" if kind == "resnets" else f"output_blocks.{idx}.1.{rest}"
    raise KeyError(f"no LDM name for UNet parameter {name}")


_VAE_RES = {"conv_shortcut": "nin_shortcut"}
_VAE_ATTN = {"group_norm": "norm", "to_q": "q", "to_k": "k", "to_v": "v", "to_out.0": "proj_out"}


def vae_ldm_name(name: str) -> str:
    """encoder + quant_conv names (the decoder is not on the training path)."""
    if name.startswith("quant_conv."):
        return name
    mod, _, leaf = name.rpartition(".")
    fixed = {"encoder.conv_in": "encoder.conv_in", "encoder.conv_norm_out": "encoder.norm_out",
             "encoder.conv_out": "encoder.conv_out"}
    if mod in fixed:
        return f"{fixed[mod]}.{leaf}"
    m = re.match(r"encoder\.down_blocks\.(\d+)\.(resnets|downsamplers)\.(\d+)\.(.*)$", name)
    if m:
        i, kind, j, rest = int(m[1]), m[2], int(m[3]), m[4]
        if kind == "downsamplers":
            return f"encoder.down.{i}.downsample.{rest}"
        head, _, lf = rest.partition(".")
        return f"encoder.down.{i}.block.{j}.{_VAE_RES.get(head, head)}.{lf}"
    m = re.match(r"encoder\.mid_block\.(resnets|attentions)\.(\d+)\.(.*)$", name)
    if m:
        kind, j, rest = m[1], int(m[2]), m[3]
        if kind == "resnets":
            return f"encoder.mid.block_{j + 1}.{rest}"
        sub, _, lf = rest.rpartition(".")
        return f"encoder.mid.attn_1.{_VAE_ATTN[sub]}.{lf}"
    raise KeyError(f"no LDM name for VAE parameter {name}")


# diffusers' deprecated attention names (AutoencoderKL._fix_state_dict_keys_on_load, used by the
# reference loader through HFModelLoaderMixin.py:117-118)
_LEGACY_VAE_ATTN = {"query": "to_q", "key": "to_k", "value": "to_v", "proj_attn": "to_out.0"}


def fix_legacy_vae_keys(sd: dict) -> dict:
    out = {}
    for k, v in sd.items():
        m = re.match(r"(.*\.attentions\.\d+)\.(query|key|value|proj_attn)\.(weight|bias)$", k)
        out[f"{m[1]}.{_LEGACY_VAE_ATTN[m[2]]}.{m[3]}" if m else k] = v
    return out


def unet_from_ldm(sd: dict, specs, cfg) -> dict:
    """diffusers-named UNet state dict out of a single-file checkpoint."""
    out = {}
    for name, shape, *_ in specs:
        key = UNET_PREFIX + unet_ldm_name(name, cfg)
        if key in sd:
            out[name] = sd[key].reshape(shape) if sd[key].numel() == _numel(shape) else sd[key]
    return out


def unet_to_ldm(sd: dict, cfg) -> dict:
    return {UNET_PREFIX + unet_ldm_name(k, cfg): v for k, v in sd.items()}


def vae_from_ldm(sd: dict, specs) -> dict:
    """diffusers-named VAE encoder state dict; LDM attention q/k/v/proj_out are 1x1 convs."""
    out = {}
    for name, shape, *_ in specs:
        key = VAE_PREFIX + vae_ldm_name(name)
        if key in sd:
            out[name] = sd[key].reshape(shape)
    return out


def vae_to_ldm(sd: dict) -> dict:
    out = {}
    for k, v in sd.items():
        ldm = vae_ldm_name(k)
        if ".mid.attn_1." in ldm and ldm.endswith(".weight") and v.dim() == 2:
            v = v.reshape(*v.shape, 1, 1)
        out[VAE_PREFIX + ldm] = v
    return out


def _numel(shape) -> int:
    n = 1
    for s in shape:
        n *= s
    return n
