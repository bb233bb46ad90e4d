"""predict / calculate_loss for SD 1.5 on the HIP kernels.

Drop-in for modules/modelSetup/BaseStableDiffusionSetup.py:135-330.  The step is the SDXL one
(BaseStableDiffusionXLSetup.py here) minus the SDXL conditioning: one text encoder whose cached
hidden state arrives as batch['text_encoder_hidden_state'] (StableDiffusionBaseDataLoader output
names), no pooled embedding and no time_ids (the SD 1.5 UNet has no add-embedding,
v1-inference.yaml:29-44).  Noise, timesteps, DDPM noising, epsilon / v-prediction targets and
the loss are the shared kernels (ModelSetupNoiseMixin / ModelSetupDiffusionMixin /
ModelSetupDiffusionLossMixin).
"""
from __future__ import annotations

import torch

from .BaseStableDiffusionXLSetup import BaseStableDiffusionXLSetup
from ..util.config.plain import plain


class BaseStableDiffusionSetup(BaseStableDiffusionXLSetup):
    def _text(self, model, batch, config, rand, B):
        """StableDiffusionModel.encode_text with cached text (StableDiffusionModel.py:188-233):
        pass-through, then the per-sample dropout mask drawn from Random(batch_seed)."""
        config = plain(config)
        te = batch["text_encoder_hidden_state"]
        p = config.text_encoder.dropout_probability
        if p is not None and p > 0:
            mask = torch.tensor([rand.random() > p for _ in range(B)], device=te.device).to(te.dtype)
            te = te * mask[:, None, None]
        return te.to(torch.bfloat16).contiguous(), None
