"""Weights from disk for the SD 1.5 / SDXL UNet, the VAE encoder and their LoRA adapters.

Load order and failure behaviour of modules/modelLoader/stableDiffusionXL/StableDiffusionXLModelLoader.py
:230-270 (the SD 1.5 loader is the same shape): INTERNAL backup (a directory with meta.json: diffusers
layout + optimizer / train progress, InternalModelLoaderMixin.py:16-42) -> diffusers directory
(`unet/`, `vae/` sub-modules, HFModelLoaderMixin.py) -> single-file .safetensors -> single-file
.ckpt (LDM layout, converted with ldm_convert.py); each failure's traceback is printed and the last
resort raises Exception("could not load model: <name>").  Text encoders (`text_encoder/`,
`text_encoder_2/`) are loaded into the caching encoders a model carries as text_encoder_1/2
(module/text_encoder.py); the train step itself consumes cached text states.
Tokenizers are host-side text processing and stay with the caller.

LoRA (modules/modelLoader/mixin/LoRALoaderMixin.py): `lora` names either an INTERNAL backup directory
(`lora/lora.safetensors` + internal data) or a .safetensors file in the reference's
LoRAModuleWrapper key layout; the state dict is handed to setup_model through
`model.lora_state_dict` like the reference.
"""
from __future__ import annotations

import json
import os
import traceback

import torch

from ..util.TrainProgress import TrainProgress
from . import ldm_convert as LC
from .HFModelLoaderMixin import TRANSFORMERS_FILES, read_diffusers_sub_module, read_single_file, read_sub_module_state_dict


def load_internal_data(model, path: str) -> None:
    """meta.json -> train_progress, optimizer/optimizer.pt -> model.optimizer_state_dict,
    ema/ema.pt -> model.ema_state_dict (weights_only loads)."""
    with open(os.path.join(path, "meta.json")) as f:
        tp = json.load(f)["train_progress"]
    model.train_progress = TrainProgress(epoch=tp["epoch"], epoch_step=tp["epoch_step"],
                                         epoch_sample=tp["epoch_sample"], global_step=tp["global_step"])
    opt = os.path.join(path, "optimizer", "optimizer.pt")
    if os.path.isfile(opt):
        model.optimizer_state_dict = torch.load(opt, map_location="cpu", weights_only=True)
    ema = os.path.join(path, "ema", "ema.pt")
    if os.path.isfile(ema):
        model.ema_state_dict = torch.load(ema, map_location="cpu", weights_only=True)


def apply_unet_state_dict(unet, sd: dict) -> None:
    """diffusers-named tensors into the flat store; every UNet parameter must be present (the
    reference's empty-weight init would leave a missing one on the meta device)."""
    missing = [n for n, *_ in unet.specs if n not in sd]
    if missing:
        raise KeyError(f"{len(missing)} UNet parameters missing, e.g. {missing[:3]}")
    unet.load_state_dict(sd)


def apply_vae_state_dict(encoder, sd: dict) -> None:
    sd = LC.fix_legacy_vae_keys(sd)
    missing = [n for n, *_ in encoder.specs if n not in sd]
    if missing:
        raise KeyError(f"{len(missing)} VAE encoder parameters missing, e.g. {missing[:3]}")
    encoder.load_state_dict({n: sd[n].reshape(shape) for n, shape, *_ in encoder.specs})


def load_vae_encoder(encoder, name: str) -> None:
    """a VAE encoder from a diffusers VAE directory (with or without a `vae/` subfolder) or a
    single-file checkpoint (`first_stage_model.*`)."""
    if os.path.isdir(name):
        for sub in ("vae", None):
            try:
                apply_vae_state_dict(encoder, read_diffusers_sub_module(name, sub))
                return
            except (FileNotFoundError, KeyError):
                continue
        raise Exception("could not load vae: " + name)
    apply_vae_state_dict(encoder, LC.vae_from_ldm(read_single_file(name), encoder.specs))


def load_text_encoder(encoder, root: str, subfolder: str) -> None:
    """a transformers text encoder (`text_encoder/`, `text_encoder_2/`: model.safetensors, sharded
    index or pytorch_model.bin) into a module.text_encoder encoder; CLIP keys without the
    `text_model.` prefix (CLIPTextModel saved by transformers 5.x) are normalised."""
    sd = read_sub_module_state_dict(root, subfolder, *TRANSFORMERS_FILES)
    names = {n for n, _ in encoder.specs}
    fixed = {}
    for k, v in sd.items():
        if k not in names and "text_model." + k in names:
            k = "text_model." + k
        fixed[k] = v
    encoder.load_state_dict(fixed)


def load_text_encoders(model, root: str, subfolders=("text_encoder", "text_encoder_2")) -> None:
    """the model's attached caching text encoders (attributes text_encoder_1 / text_encoder_2), if any."""
    for attr, sub in zip(("text_encoder_1", "text_encoder_2"), subfolders):
        enc = getattr(model, attr, None)
        if enc is not None:
            load_text_encoder(enc, root, sub)


class StableDiffusionXLModelLoader:
    """also serves SD 1.5 (the UNet config on the model decides the key layout)."""

    def _load_diffusers(self, model, base: str, vae: str | None):
        apply_unet_state_dict(model.unet, read_diffusers_sub_module(base, "unet"))
        load_text_encoders(model, base)
        enc = getattr(model, "vae_encoder", None)
        if enc is not None:
            load_vae_encoder(enc, vae or base)

    def _load_internal(self, model, base: str, vae: str | None):
        if not os.path.isfile(os.path.join(base, "meta.json")):
            raise Exception("not an internal model")
        self._load_diffusers(model, base, vae)
        load_internal_data(model, base)

    def _load_single_file(self, model, base: str, vae: str | None, ext: str):
        if not base.endswith(ext):
            raise Exception(f"not a {ext} file")
        sd = read_single_file(base)
        apply_unet_state_dict(model.unet, LC.unet_from_ldm(sd, model.unet.specs, model.unet.cfg))
        enc = getattr(model, "vae_encoder", None)
        if enc is not None:
            if vae:
                load_vae_encoder(enc, vae)
            else:
                apply_vae_state_dict(enc, LC.vae_from_ldm(sd, enc.specs))

    def load(self, model, model_names) -> None:
        base, vae = model_names.base_model, model_names.vae_model or None
        stacktraces = []
        for fn in (lambda: self._load_internal(model, base, vae), lambda: self._load_diffusers(model, base, vae),
                   lambda: self._load_single_file(model, base, vae, ".safetensors"),
                   lambda: self._load_single_file(model, base, vae, ".ckpt")):
            try:
                fn()
                return
            except Exception:
                stacktraces.append(traceback.format_exc())
        for st in stacktraces:
            print(st)
        raise Exception("could not load model: " + base)


class StableDiffusionXLLoRAModelLoader:
    """base weights (optional: an empty base name keeps the random init) + adapter state."""

    def load(self, model, model_names) -> None:
        if model_names.base_model:
            StableDiffusionXLModelLoader().load(model, model_names)
        lora = model_names.lora
        if not lora:
            return
        if os.path.isdir(lora):
            if not os.path.isfile(os.path.join(lora, "meta.json")):
                raise Exception("could not load LoRA: " + lora)
            model.lora_state_dict = read_single_file(os.path.join(lora, "lora", "lora.safetensors"))
            load_internal_data(model, lora)
        else:
            model.lora_state_dict = read_single_file(lora)
