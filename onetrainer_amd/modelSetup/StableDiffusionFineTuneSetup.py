"""SD 1.5 full fine-tune plugin (mirrors modules/modelSetup/StableDiffusionFineTuneSetup.py):
the SDXL fine-tune plugin's parameter groups / fused AdamW over the SD 1.5 step."""
from __future__ import annotations

from .BaseStableDiffusionSetup import BaseStableDiffusionSetup
from .StableDiffusionXLFineTuneSetup import StableDiffusionXLFineTuneSetup


class StableDiffusionFineTuneSetup(BaseStableDiffusionSetup, StableDiffusionXLFineTuneSetup):
    pass
