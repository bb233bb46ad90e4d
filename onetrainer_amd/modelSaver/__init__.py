"""Writing models and backups, in the layouts the reference writes:

  * DIFFUSERS (modules/modelSaver/stableDiffusionXL/StableDiffusionXLModelSaver.py:22-42): a directory
    with `unet/` (or `transformer/`) `diffusion_pytorch_model.safetensors` + `config.json`, sharded
    with an index at 10 GB like save_pretrained's default, and `model_index.json`;
  * SAFETENSORS (:44-67): one file in the LDM layout (`model.diffusion_model.*`, `first_stage_model.*`
    when a VAE encoder is attached) plus the noise-schedule buffers of
    convert_diffusers_to_ckpt_util.map_noise_scheduler and `v_pred` for v-prediction;
  * INTERNAL (backups, :69-74 + InternalModelSaverMixin.py:14-42): the DIFFUSERS layout (LoRA:
    `lora/lora.safetensors`) plus `optimizer/optimizer.pt` (state dict + param_group_mapping +
    param_group_optimizer_mapping), `ema/ema.pt` when an EMA exists, and `meta.json` with the
    train progress.
Tensors are written from the device copy of each parameter (diffusers layout: NCHW convs, unpadded).
LoRA files keep the LoRAModuleWrapper key layout (the OMI key conversion lives in the absent
omi_model_standards package).
"""
from __future__ import annotations

import json
import os

import torch
from safetensors.torch import save_file

from ..modelLoader import ldm_convert as LC

MAX_SHARD_BYTES = 10 * 10 ** 9


def _cpu(sd: dict, dtype=None) -> dict:
    return {k: (v.to(dtype) if dtype is not None and v.is_floating_point() else v).detach().cpu().contiguous()
            for k, v in sd.items()}


def save_sub_module(sd: dict, dest: str, config: dict | None = None, max_shard_bytes: int = MAX_SHARD_BYTES) -> None:
    os.makedirs(dest, exist_ok=True)
    if config is not None:
        with open(os.path.join(dest, "config.json"), "w") as f:
            json.dump(config, f, indent=2)
    total = sum(v.numel() * v.element_size() for v in sd.values())
    if total <= max_shard_bytes:
        save_file(sd, os.path.join(dest, "diffusion_pytorch_model.safetensors"))
        return
    shards, cur, size = [], {}, 0
    for k, v in sd.items():
        nb = v.numel() * v.element_size()
        if cur and size + nb > max_shard_bytes:
            shards.append(cur)
            cur, size = {}, 0
        cur[k] = v
        size += nb
    shards.append(cur)
    weight_map = {}
    for i, sh in enumerate(shards):
        name = f"diffusion_pytorch_model-{i + 1:05d}-of-{len(shards):05d}.safetensors"
        save_file(sh, os.path.join(dest, name))
        weight_map |= {k: name for k in sh}
    with open(os.path.join(dest, "diffusion_pytorch_model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {"total_size": total}, "weight_map": weight_map}, f, indent=2)


def schedule_buffers(betas: torch.Tensor) -> dict:
    """DiffusionScheduleCoefficients.from_betas (modules/util/DiffusionScheduleCoefficients.py:37-60),
    the buffers a single-file SD checkpoint carries."""
    betas = betas.float().cpu()
    acp = torch.cumprod(1 - betas, dim=0)
    acp_prev = torch.cat((torch.ones(1), acp[:-1]))
    post_var = betas * (1 - acp_prev) / (1 - acp)
    return {"betas": betas, "alphas_cumprod": acp, "alphas_cumprod_prev": acp_prev,
            "sqrt_alphas_cumprod": acp.sqrt(), "sqrt_one_minus_alphas_cumprod": (1 - acp).sqrt(),
            "log_one_minus_alphas_cumprod": (1 - acp).log(), "sqrt_recip_alphas_cumprod": acp.rsqrt(),
            "sqrt_recipm1_alphas_cumprod": (1 / acp - 1).sqrt(), "posterior_variance": post_var,
            "posterior_log_variance_clipped": torch.cat([post_var[1:2], post_var[1:]]).clamp(min=1e-20).log()}


def unet_diffusers_config(cfg) -> dict:
    """the UNet2DConditionModel config fields the architecture is pinned by (sd_xl_base.yaml:19-37,
    v1-inference.yaml:29-44)."""
    heads = cfg.num_heads if cfg.num_heads else [c // cfg.head_dim for c in cfg.block_out_channels]
    return {"_class_name": "UNet2DConditionModel", "in_channels": cfg.in_channels, "out_channels": cfg.out_channels,
            "block_out_channels": list(cfg.block_out_channels), "down_block_types": list(cfg.down_block_types),
            "up_block_types": list(cfg.up_block_types), "layers_per_block": cfg.layers_per_block,
            "transformer_layers_per_block": list(cfg.transformer_layers_per_block),
            "attention_head_dim": heads, "cross_attention_dim": cfg.cross_attention_dim,
            "use_linear_projection": cfg.use_linear_projection, "norm_num_groups": cfg.norm_num_groups,
            "norm_eps": cfg.norm_eps,
            "addition_embed_type": "text_time" if cfg.addition_embed else None,
            "addition_time_embed_dim": cfg.addition_time_embed_dim if cfg.addition_embed else None,
            "projection_class_embeddings_input_dim":
                cfg.projection_class_embeddings_input_dim if cfg.addition_embed else None}


def save_internal_data(model, config, dest: str) -> None:
    os.makedirs(os.path.join(dest, "optimizer"), exist_ok=True)
    sd = model.optimizer.state_dict()
    sd["param_group_mapping"] = list(model.param_group_mapping)
    sd["param_group_optimizer_mapping"] = [str(config.optimizer.optimizer) for _ in model.param_group_mapping]
    torch.save(sd, os.path.join(dest, "optimizer", "optimizer.pt"))
    if getattr(model, "ema", None) is not None:
        os.makedirs(os.path.join(dest, "ema"), exist_ok=True)
        torch.save(model.ema.state_dict(), os.path.join(dest, "ema", "ema.pt"))
    tp = model.train_progress
    with open(os.path.join(dest, "meta.json"), "w") as f:
        json.dump({"train_progress": {"epoch": tp.epoch, "epoch_step": tp.epoch_step, "epoch_sample": tp.epoch_sample,
                                      "global_step": tp.global_step}}, f)


class StableDiffusionXLModelSaver:
    """fine-tune saver for SD 1.5 / SDXL."""

    def save(self, model, config, output_model_format: str, dest: str, dtype=None) -> None:
        unet_sd = _cpu(model.unet.state_dict(), dtype)
        enc = getattr(model, "vae_encoder", None)
        if output_model_format in ("DIFFUSERS", "INTERNAL"):
            os.makedirs(dest, exist_ok=True)
            save_sub_module(unet_sd, os.path.join(dest, "unet"), unet_diffusers_config(model.unet.cfg))
            if enc is not None:
                save_sub_module(_cpu(enc.state_dict(), dtype), os.path.join(dest, "vae"),
                                {"_class_name": "AutoencoderKL", "scaling_factor": enc.cfg.scaling_factor})
            with open(os.path.join(dest, "model_index.json"), "w") as f:
                json.dump({"_class_name": "StableDiffusionXLPipeline" if model.unet.cfg.addition_embed
                           else "StableDiffusionPipeline", "unet": ["diffusers", "UNet2DConditionModel"]}, f)
            if output_model_format == "INTERNAL":
                save_internal_data(model, config, dest)
            return
        if output_model_format == "SAFETENSORS":
            sd = LC.unet_to_ldm(unet_sd, model.unet.cfg)
            if enc is not None:
                sd |= LC.vae_to_ldm(_cpu(enc.state_dict(), dtype))
            sd |= schedule_buffers(model.noise_scheduler.betas)
            if model.noise_scheduler.config.prediction_type == "v_prediction":
                sd["v_pred"] = torch.tensor([])
            os.makedirs(os.path.dirname(os.path.abspath(dest)), exist_ok=True)
            save_file(sd, dest)
            return
        raise NotImplementedError(f"output format {output_model_format}")


class LoRAModelSaver:
    """adapters of `model.<lora_attr>` (SDXL: unet_lora, Flux: transformer_lora)."""

    def __init__(self, lora_attr: str):
        self.lora_attr = lora_attr

    def save(self, model, config, output_model_format: str, dest: str, dtype=None) -> None:
        sd = _cpu(getattr(model, self.lora_attr).state_dict(), dtype)
        if output_model_format == "SAFETENSORS":
            os.makedirs(os.path.dirname(os.path.abspath(dest)), exist_ok=True)
            save_file(sd, dest)
            return
        if output_model_format == "INTERNAL":
            os.makedirs(os.path.join(dest, "lora"), exist_ok=True)
            save_file(sd, os.path.join(dest, "lora", "lora.safetensors"))
            save_internal_data(model, config, dest)
            return
        raise NotImplementedError(f"output format {output_model_format} for LoRA")


class FluxModelSaver:
    def save(self, model, config, output_model_format: str, dest: str, dtype=None) -> None:
        if output_model_format not in ("DIFFUSERS", "INTERNAL"):
            raise NotImplementedError(f"output format {output_model_format} for FLUX fine-tunes")
        c = model.transformer.cfg
        save_sub_module(_cpu(model.transformer.state_dict(), dtype), os.path.join(dest, "transformer"),
                        {"_class_name": "FluxTransformer2DModel", "num_layers": c.num_layers,
                         "num_single_layers": c.num_single_layers, "attention_head_dim": c.attention_head_dim,
                         "num_attention_heads": c.num_attention_heads, "joint_attention_dim": c.joint_attention_dim,
                         "pooled_projection_dim": c.pooled_projection_dim, "in_channels": c.in_channels,
                         "guidance_embeds": c.guidance_embeds, "axes_dims_rope": list(c.axes_dims_rope)})
        with open(os.path.join(dest, "model_index.json"), "w") as f:
            json.dump({"_class_name": "FluxPipeline", "transformer": ["diffusers", "FluxTransformer2DModel"]}, f)
        if output_model_format == "INTERNAL":
            save_internal_data(model, config, dest)


def create_model_saver(model_type: str, training_method: str):
    """ModelType x TrainingMethod -> saver (modules/util/create.py create_model_saver)."""
    flux = model_type.startswith("FLUX")
    if training_method == "LORA":
        return LoRAModelSaver("transformer_lora" if flux else "unet_lora")
    return FluxModelSaver() if flux else StableDiffusionXLModelSaver()
