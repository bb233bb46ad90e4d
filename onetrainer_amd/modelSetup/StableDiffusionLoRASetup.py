"""SD 1.5 LoRA plugin (mirrors modules/modelSetup/StableDiffusionLoRASetup.py): frozen bf16 UNet,
fp32 adapters (module/lora.py), over the SD 1.5 step."""
from __future__ import annotations

from .BaseStableDiffusionSetup import BaseStableDiffusionSetup
from .StableDiffusionXLLoRASetup import StableDiffusionXLLoRASetup


class StableDiffusionLoRASetup(BaseStableDiffusionSetup, StableDiffusionXLLoRASetup):
    pass
