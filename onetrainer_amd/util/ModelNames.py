"""Which weights to load (mirrors modules/util/ModelNames.py for the parts the hot path loads)."""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class ModelNames:
    base_model: str = ""
    vae_model: str = ""
    lora: str = ""
