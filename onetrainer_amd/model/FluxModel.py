"""Model container for FLUX.1 training (mirrors the attribute bag of modules/model/FluxModel.py that the
setup and trainer read: transformer, noise_scheduler, vae.config (scaling / shift factor), train_dtype,
optimizer, transformer_lora, train_progress)."""
from __future__ import annotations

from types import SimpleNamespace

import torch

from ..util.TrainProgress import TrainProgress
from .StableDiffusionXLModel import AttrDict


class FlowMatchScheduler:
    """the parts of FlowMatchEulerDiscreteScheduler the reference reads on the hot path
    (config.num_train_timesteps; timesteps / sigmas only for their length, ModelSetupFlowMatchingMixin.py:14-39)."""

    def __init__(self, num_train_timesteps=1000):
        self.config = AttrDict(num_train_timesteps=num_train_timesteps)
        self.timesteps = torch.arange(num_train_timesteps, 0, -1, dtype=torch.float32)
        self.sigmas = self.timesteps / num_train_timesteps


class FluxModel:
    def __init__(self, transformer, noise_scheduler=None, vae_scaling_factor=0.3611, vae_shift_factor=0.1159,
                 model_type="FLUX_DEV_1"):
        self.model_type = model_type
        self.transformer = transformer
        self.noise_scheduler = noise_scheduler or FlowMatchScheduler()
        self.vae = SimpleNamespace(config={"scaling_factor": vae_scaling_factor, "shift_factor": vae_shift_factor})
        self.train_dtype = torch.bfloat16
        self.optimizer = None
        self.param_group_mapping = None
        self.parameters = None
        self.ema = None
        self.train_progress = TrainProgress()
        self.transformer_lora = None

    @property
    def train_store(self):
        return self.transformer_lora.store if self.transformer_lora is not None else self.transformer.store
