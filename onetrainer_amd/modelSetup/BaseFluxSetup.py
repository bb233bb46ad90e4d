"""predict / calculate_loss for FLUX.1 on the HIP kernels.

Drop-in for modules/modelSetup/BaseFluxSetup.py:193-390 with the math of ModelSetupNoiseMixin
(noise; LOGIT_NORMAL / UNIFORM timesteps, static or dynamic shift), ModelSetupFlowMatchingMixin.py:14-39
(sigma = (t + 1) / N, x_t = sigma noise + (1 - sigma) x0), FluxModel.pack/unpack_latents and
ModelSetupDiffusionLossMixin._flow_matching_losses (unmasked MSE, flow target noise - x0):
  * latents arrive [B, 16, h, w] (this build's loaders: a view of channels-last storage);
  * one prologue kernel does the shift / scale, the noising and the flow target;
  * the transformer gets t / 1000 and guidance = prior.guidance_scale, like the reference.
Batch contract: text_encoder_1_pooled_state [B, 768] (CLIP pooled), text_encoder_2_hidden_state
[B, L, 4096] (T5), latent_image, loss_weight (FluxBaseDataLoader output names).
"""
from __future__ import annotations

import math
from random import Random

import torch

from .. import kernels as K
from ..module import flux_ops as O
from ..module import functional as Fn
from .BaseStableDiffusionXLSetup import draw_noise, loss_plan, nhwc_pair, report_learning_rates, timestep_plan
from ..util.config.plain import plain


class BaseFluxSetup:
    def __init__(self, train_device, temp_device=None, debug_mode=False, dp_rank=0, dp_world=1):
        self.train_device = torch.device(train_device)
        self.temp_device = temp_device
        self.debug_mode = debug_mode
        self.dp_rank = dp_rank
        self.dp_world = dp_world
        self.graph_inputs = None   # injected (noise NHWC, timestep int32): parity tests

    @staticmethod
    def _nhwc_latent(lat: torch.Tensor) -> torch.Tensor:
        """[B, 16, h, w] (reference contract; channels-last storage from this build's loaders) -> NHWC."""
        return lat.permute(0, 2, 3, 1).contiguous()

    def _text(self, batch, config, rand, B):
        """FluxModel.encode_text with cached outputs: per-encoder dropout masks from Random(seed)."""
        config = plain(config)
        pooled = batch["text_encoder_1_pooled_state"]
        ehs = batch["text_encoder_2_hidden_state"]
        p1, p2 = config.text_encoder.dropout_probability, config.text_encoder_2.dropout_probability
        if p1 is not None and p1 > 0:
            m = torch.tensor([rand.random() > p1 for _ in range(B)], device=pooled.device).to(pooled.dtype)
            pooled = pooled * m[:, None]
        if p2 is not None and p2 > 0:
            m = torch.tensor([rand.random() > p2 for _ in range(B)], device=ehs.device).to(ehs.dtype)
            ehs = ehs * m[:, None, None]
        return pooled.to(torch.bfloat16).contiguous(), ehs.to(torch.bfloat16).contiguous()

    def report_to_tensorboard(self, model, config, lr_scheduler, tensorboard):
        report_learning_rates(model, lr_scheduler, tensorboard)

    def _shift(self, config, h, w):
        """ModelSetupNoiseMixin._get_timestep_discrete: static timestep_shift, or the dynamic one of the
        image sequence length (base 256 -> 0.5, max 4096 -> 1.15, patch 2)."""
        config = plain(config)
        if not config.dynamic_timestep_shifting:
            return config.timestep_shift
        m = (1.15 - 0.5) / (4096 - 256)
        mu = (w // 2) * (h // 2) * m + (0.5 - m * 256)
        return math.exp(mu)

    def predict(self, model, batch: dict, config, train_progress, *, deterministic: bool = False) -> dict:
        config = plain(config)
        batch_seed = 0 if deterministic else train_progress.global_step
        rand = Random(batch_seed)
        latent = self._nhwc_latent(batch["latent_image"])
        B, h, w, C = latent.shape
        pooled, ehs = self._text(batch, config, rand, B)
        N = model.noise_scheduler.config["num_train_timesteps"]
        if self.graph_inputs is not None:
            noise, timestep = self.graph_inputs
        else:
            sample0 = self.dp_rank * B
            noise = draw_noise(config, latent.shape, batch_seed, sample0 * h * w * C, latent.dtype, latent.device)
            if deterministic:
                timestep = torch.full((B,), int(N * 0.5) - 1, dtype=torch.int32, device=latent.device)
            else:
                timestep = K.timesteps(B, seed=batch_seed, sample0=sample0, dist=timestep_plan(config),
                                       num_train_timesteps=N, min_s=config.min_noising_strength, max_s=config.max_noising_strength,
                                       shift=self._shift(config, h, w), bias=config.noising_bias,
                                       weight=config.noising_weight, device=latent.device)
        vc = model.vae.config
        model_in, target = K.flow_prologue(latent, noise, timestep, vc["scaling_factor"], vc["shift_factor"], N,
                                           cpad=C)
        tokens = K.flux_pack(model_in)
        guidance = None
        if model.transformer.config["guidance_embeds"]:
            guidance = torch.full((B,), float(config.prior.guidance_scale), dtype=torch.float32, device=latent.device)
        # timestep / 1000 (BaseFluxSetup.py:291) as an IEEE division: torch's tensor / python-scalar on the GPU
        # multiplies by the reciprocal (1 ulp off in places); a tensor divisor divides
        t_model = timestep.float() / torch.full((B,), 1000.0, dtype=torch.float32, device=latent.device)
        pred_tok = model.transformer(tokens, t_model, guidance, pooled, ehs, h, w)
        pred = O.UnpackFn.apply(pred_tok, B, h, w, C)
        # reference contract: [B, 16, h, w] (BaseFluxSetup.py:301-307); views of the NHWC kernel tensors
        return {"loss_type": "target", "timestep": timestep, "predicted": pred.permute(0, 3, 1, 2),
                "target": target.permute(0, 3, 1, 2), "_predicted_nhwc": pred, "_target_nhwc": target}

    def calculate_loss(self, model, batch: dict, data: dict, config) -> torch.Tensor:
        """_flow_matching_losses(...).mean() (BaseFluxSetup.py:377-390): unmasked MSE x loss_weight x scalers."""
        plan = loss_plan(plain(config), flow=True)
        lw = batch.get("loss_weight")
        lw = lw.to(self.train_device, torch.float32).contiguous() if lw is not None else None
        pred, target = nhwc_pair(data, 16)
        N = model.noise_scheduler.config["num_train_timesteps"]
        return Fn.MSELossFn.apply(pred, target, lw, data["timestep"], None, plan["loss_fn"], plan["gamma"], False, 1.0,
                                  plan["mse_strength"], float(plan["batch_size_scale"] * plan["ga_scale"]),
                                  1.0 / self.dp_world, N)
