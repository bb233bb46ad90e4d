"""Synthetic cached-latent batches in the reference's batch contract
(DataLoaderText2ImageMixin._output_modules_from_out_names, DataLoaderText2ImageMixin.py:248-294;
SDXL names StableDiffusionXLBaseDataLoader.py:174-209) for benchmarks and tests.

latent ~ N(0,1)/scaling_factor (so the scaled latent is N(0,1)), text states ~ N(0,1),
time_ids = (H, W, 0, 0, H, W), loss_weight = 1, concept_type 'STANDARD' (SURVEY.md §8(d)).
Latents are produced NHWC [B,h,w,4] (this build's layout).  `resident=True` keeps one batch in
HBM and re-yields it (bench: inputs already resident when the timed region starts)."""
from __future__ import annotations

import torch


def synthetic_sdxl_batch(batch_size, height, width, device, seed=0, latent_dtype=torch.float32,
                         scaling_factor=0.13025, te1_dim=768, te2_dim=1280, pooled_dim=1280, text_len=77,
                         sdxl=True):
    g = torch.Generator(device="cpu").manual_seed(seed)
    h, w = height // 8, width // 8
    lat = (torch.randn(batch_size, h, w, 4, generator=g) / scaling_factor).to(device, latent_dtype)
    b = {
        "latent_image": lat.permute(0, 3, 1, 2),   # the reference's NCHW contract, channels-last storage
        "text_encoder_1_hidden_state": torch.randn(batch_size, text_len, te1_dim, generator=g).to(device, torch.bfloat16),
        "loss_weight": torch.ones(batch_size, device=device),
        "concept_type": ["STANDARD"] * batch_size,
    }
    if sdxl:
        b["text_encoder_2_hidden_state"] = torch.randn(batch_size, text_len, te2_dim, generator=g).to(device, torch.bfloat16)
        b["text_encoder_2_pooled_state"] = torch.randn(batch_size, pooled_dim, generator=g).to(device, torch.bfloat16)
        hw = lambda v: torch.full((batch_size,), v, dtype=torch.int64, device=device)
        b["original_resolution"] = (hw(height), hw(width))
        b["crop_offset"] = (hw(0), hw(0))
        b["crop_resolution"] = (hw(height), hw(width))
    else:   # SD 1.5 output names (StableDiffusionBaseDataLoader): one text encoder
        b["text_encoder_hidden_state"] = b.pop("text_encoder_1_hidden_state")
    return b


class SyntheticDataLoader:
    def __init__(self, batch_size, height, width, device, steps_per_epoch=100, seed=0, resident=True, sdxl=True):
        self.batch_size, self.height, self.width, self.device = batch_size, height, width, device
        self.steps_per_epoch, self.seed, self.resident, self.sdxl = steps_per_epoch, seed, resident, sdxl
        self._batch = None

    def approximate_length(self):
        return self.steps_per_epoch

    def start_next_epoch(self):
        pass

    def get_data_set(self):
        return self

    def get_data_loader(self):
        for i in range(self.steps_per_epoch):
            if self.resident:
                if self._batch is None:
                    self._batch = synthetic_sdxl_batch(self.batch_size, self.height, self.width, self.device,
                                                       self.seed, sdxl=self.sdxl)
                yield self._batch
            else:
                yield synthetic_sdxl_batch(self.batch_size, self.height, self.width, self.device, self.seed + i,
                                           sdxl=self.sdxl)


def synthetic_flux_batch(batch_size, height, width, device, seed=0, latent_dtype=torch.float32, channels=16,
                         scaling_factor=0.3611, shift_factor=0.1159, t5_dim=4096, pooled_dim=768, text_len=77):
    """Flux output names (FluxBaseDataLoader): latent ~ N(0,1)/sf + shift so the scaled latent is N(0,1)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    h, w = height // 8, width // 8
    lat = (torch.randn(batch_size, h, w, channels, generator=g) / scaling_factor + shift_factor).to(device, latent_dtype)
    return {
        "latent_image": lat.permute(0, 3, 1, 2),   # NCHW view of channels-last storage
        "text_encoder_1_pooled_state": torch.randn(batch_size, pooled_dim, generator=g).to(device, torch.bfloat16),
        "text_encoder_2_hidden_state": torch.randn(batch_size, text_len, t5_dim, generator=g).to(device, torch.bfloat16),
        "loss_weight": torch.ones(batch_size, device=device),
        "concept_type": ["STANDARD"] * batch_size,
    }
