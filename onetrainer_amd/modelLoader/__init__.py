"""Model weights from disk: diffusers directories, single files, INTERNAL backups."""
from __future__ import annotations


def create_model_loader(model_type: str, training_method: str):
    """ModelType x TrainingMethod -> loader (modules/util/create.py create_model_loader)."""
    lora = training_method == "LORA"
    if model_type.startswith("FLUX"):
        from .FluxModelLoader import FluxLoRAModelLoader, FluxModelLoader
        return FluxLoRAModelLoader() if lora else FluxModelLoader()
    if model_type.startswith("STABLE_DIFFUSION"):
        from .StableDiffusionModelLoader import StableDiffusionXLLoRAModelLoader, StableDiffusionXLModelLoader
        return StableDiffusionXLLoRAModelLoader() if lora else StableDiffusionXLModelLoader()
    raise NotImplementedError(f"model type {model_type}")
