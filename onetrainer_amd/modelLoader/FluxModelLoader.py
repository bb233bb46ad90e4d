"""FLUX.1 transformer weights from a local diffusers directory (`transformer/`, sharded or not) or an
INTERNAL backup; the same order and failure message as modules/modelLoader/flux/FluxModelLoader.py
(internal -> diffusers; the single-file BFL layout needs diffusers' converter and is not restated).
LoRA: `lora/lora.safetensors` of a backup or a .safetensors file (LoRAModuleWrapper keys).
When the trainer caches latents / text it attaches the 16-channel VAE encoder and the CLIP-L / T5-XXL encoders
first (dataLoader/create.attach_cache_encoders); they are filled from `vae/`, `text_encoder/`, `text_encoder_2/`."""
from __future__ import annotations

import os
import traceback

from .HFModelLoaderMixin import read_diffusers_sub_module, read_single_file
from .StableDiffusionModelLoader import load_internal_data, load_text_encoders, load_vae_encoder


def apply_flux_state_dict(transformer, sd: dict) -> None:
    missing = [n for n, *_ in transformer.specs if n not in sd]
    if missing:
        raise KeyError(f"{len(missing)} transformer parameters missing, e.g. {missing[:3]}")
    transformer.load_state_dict(sd)


class FluxModelLoader:
    def load(self, model, model_names) -> None:
        base = model_names.base_model
        stacktraces = []
        try:
            if not os.path.isfile(os.path.join(base, "meta.json")):
                raise Exception("not an internal model")
            apply_flux_state_dict(model.transformer, read_diffusers_sub_module(base, "transformer"))
            load_internal_data(model, base)
            return
        except Exception:
            stacktraces.append(traceback.format_exc())
        try:
            apply_flux_state_dict(model.transformer, read_diffusers_sub_module(base, "transformer"))
            load_text_encoders(model, base)
            enc = getattr(model, "vae_encoder", None)
            if enc is not None:
                load_vae_encoder(enc, getattr(model_names, "vae_model", None) or base)
            return
        except Exception:
            stacktraces.append(traceback.format_exc())
        for st in stacktraces:
            print(st)
        raise Exception("could not load model: " + base)


class FluxLoRAModelLoader:
    def load(self, model, model_names) -> None:
        if model_names.base_model:
            FluxModelLoader().load(model, model_names)
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
