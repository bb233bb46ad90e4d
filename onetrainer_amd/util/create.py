"""Factories (mirrors the parts of modules/util/create.py the hot path uses:
create_model_setup 285-353, create_optimizer 509-534 via setup_model, create_lr_scheduler
1114-1232, create_noise_scheduler 1235-1373)."""
from __future__ import annotations

import torch

from ..model.StableDiffusionXLModel import NoiseScheduler, StableDiffusionXLModel
from ..module import unet as U
from ..util.lr_scheduler_util import create_lr_scheduler  # noqa: F401  (re-export)
from .config.plain import plain

SCALING = {"STABLE_DIFFUSION_XL_10_BASE": 0.13025, "STABLE_DIFFUSION_15": 0.18215}


def is_flux(model_type: str) -> bool:
    return model_type.startswith("FLUX")


def create_model(config, device, seed=0, unet_config=None, prediction_type="epsilon", flux_config=None):
    """random-weight model of the configured architecture (weights from disk: SURVEY.md §8(f) #2).
    LoRA training keeps the base network frozen (no gradient buffer)."""
    from .dtype_util import dtype_plan
    config = plain(config)
    plan = dtype_plan(config)   # ValueError for a dtype setup the build cannot train, before any allocation
    mt = config.model_type
    if is_flux(mt):
        from ..model.FluxModel import FluxModel
        from ..module import flux as FX
        tr = FX.FluxTransformer2DModel(flux_config or FX.flux_dev_config(), device, seed=seed,
                                       trainable=config.training_method != "LORA", master=plan.master)
        m = FluxModel(tr, model_type=mt)
        m.dtype_plan = plan
        return m
    if unet_config is None:
        unet_config = _unet_config_on_disk(config)
    if unet_config is None:
        if mt.startswith("STABLE_DIFFUSION_XL"):
            unet_config = U.sdxl_config()
        elif is_sd15(mt):
            unet_config = U.sd15_config()
        else:
            raise NotImplementedError(f"model type {mt}")
    unet = U.UNet2DConditionModel(unet_config, device, seed=seed, trainable=config.training_method != "LORA",
                                  master=plan.master)
    ns = NoiseScheduler(device, prediction_type=prediction_type)
    m = StableDiffusionXLModel(unet, ns, SCALING.get(mt, 0.13025), model_type=mt)
    m.dtype_plan = plan
    return m


def _unet_config_on_disk(config):
    """the architecture a diffusers-layout model directory declares (`unet/config.json`, as
    diffusers' from_pretrained reads it): the backup continued from, else base_model_name.
    Single-file checkpoints carry no config and keep the model type's architecture."""
    import json
    import os
    names = []
    if getattr(config, "continue_last_backup", False) and config.training_method != "LORA":
        last = config.get_last_backup_path() if hasattr(config, "get_last_backup_path") else None
        names.append(last)
    names.append(getattr(config, "base_model_name", None))
    for name in names:
        path = os.path.join(name, "unet", "config.json") if name else None
        if path and os.path.isfile(path):
            with open(path) as f:
                return U.unet_config_from_diffusers(json.load(f))
    return None


def is_sd15(model_type: str) -> bool:
    return model_type.startswith("STABLE_DIFFUSION_15") or model_type in ("STABLE_DIFFUSION_15_INPAINTING",)


def create_model_setup(config, train_device, dp_rank=0, dp_world=1):
    """ModelType x TrainingMethod -> plugin (create.py:285-353)."""
    config = plain(config)
    if is_flux(config.model_type):
        if config.training_method == "LORA":
            from ..modelSetup.FluxLoRASetup import FluxLoRASetup as S
        elif config.training_method == "FINE_TUNE":
            from ..modelSetup.FluxFineTuneSetup import FluxFineTuneSetup as S
        else:
            raise NotImplementedError(f"training method {config.training_method}")
        return S(train_device, dp_rank=dp_rank, dp_world=dp_world)
    sd15 = is_sd15(config.model_type)
    if not sd15 and not config.model_type.startswith("STABLE_DIFFUSION_XL"):
        raise NotImplementedError(f"model type {config.model_type}")
    if config.training_method == "FINE_TUNE":
        if sd15:
            from ..modelSetup.StableDiffusionFineTuneSetup import StableDiffusionFineTuneSetup as S
        else:
            from ..modelSetup.StableDiffusionXLFineTuneSetup import StableDiffusionXLFineTuneSetup as S
        return S(train_device, dp_rank=dp_rank, dp_world=dp_world)
    if config.training_method == "LORA":
        if sd15:
            from ..modelSetup.StableDiffusionLoRASetup import StableDiffusionLoRASetup as S
        else:
            from ..modelSetup.StableDiffusionXLLoRASetup import StableDiffusionXLLoRASetup as S
        return S(train_device, dp_rank=dp_rank, dp_world=dp_world)
    raise NotImplementedError(f"training method {config.training_method}")
