"""predict / calculate_loss for SDXL (and SD1.5: no add-embedding) on the HIP kernels.

Drop-in for modules/modelSetup/BaseStableDiffusionXLSetup.py:179-373 (predict, calculate_loss),
with the math of ModelSetupNoiseMixin.py:18-155, ModelSetupDiffusionMixin.py:15-38 and
ModelSetupDiffusionLossMixin.py:119-279 done by csrc/diffusion.hip:
  * noise / timesteps: Philox, seeded by the same `batch_seed` (0 if deterministic else
    global_step); counter = index in the GLOBAL batch, so DP rank r draws exactly its slice;
  * DDPM noising + target (epsilon / v_prediction) in one prologue kernel;
  * unmasked MSE (+ MIN_SNR_GAMMA / DEBIASED_ESTIMATION / P2 weights, loss_weight, scalers).
Batch contract as the reference's data loader (StableDiffusionXLBaseDataLoader.py:174-209),
with `latent_image` [B, 4, h, w]; this build's loaders hand it over as a view of channels-last
storage, so the kernels' NHWC layout costs no copy.
"""
from __future__ import annotations

from random import Random

import torch

from .. import kernels as K
from ..module import functional as Fn
from ..util.config.plain import plain

LOSS_FN = {"CONSTANT": 0, "MIN_SNR_GAMMA": 1, "DEBIASED_ESTIMATION": 2, "P2": 3}
TIMESTEP_DIST = {"UNIFORM": 0, "LOGIT_NORMAL": 1}


def loss_plan(config, flow: bool = False) -> dict:
    """The loss decisions of ModelSetupDiffusionLossMixin for this config (config already plain()):
    batch / GA scale (LossScaler, :243-248 / :290-295) and the timestep weight kernel id (:271-278 for
    DDPM: MIN_SNR_GAMMA / DEBIASED_ESTIMATION / P2, anything else unweighted; :316-319 for flow
    matching: SIGMA, anything else unweighted)."""
    if config.mae_strength != 0 or config.log_cosh_strength != 0 or config.masked_training:
        raise NotImplementedError("only the unmasked MSE loss of C1-C5 is on this build's hot path")
    scaler = config.loss_scaler
    if scaler not in ("NONE", "BATCH", "GRADIENT_ACCUMULATION", "BOTH"):
        raise ValueError(f"loss_scaler {scaler!r}")
    bs = 1 if scaler in ("NONE", "GRADIENT_ACCUMULATION") else config.batch_size
    gas = 1 if scaler in ("NONE", "BATCH") else config.gradient_accumulation_steps
    fn = config.loss_weight_fn
    if flow:
        kid = 4 if fn == "SIGMA" else 0
    else:
        kid = LOSS_FN.get(fn, 0)
    return {"batch_size_scale": bs, "ga_scale": gas, "loss_fn": kid, "gamma": float(config.loss_weight_strength),
            "mse_strength": float(config.mse_strength)}


def timestep_plan(config) -> int:
    """kernel id of config.timestep_distribution (ModelSetupNoiseMixin.py:91-118); the discrete
    SIGMOID / COS_MAP / HEAVY_TAIL samplers are outside C1-C5."""
    d = config.timestep_distribution
    if d not in TIMESTEP_DIST:
        raise NotImplementedError(f"timestep distribution {d} is not on this build's hot path")
    return TIMESTEP_DIST[d]


def draw_noise(config, shape, seed, offset, dtype, device, out=None):
    """_create_noise (ModelSetupNoiseMixin.py:18-49) for an NHWC latent: Philox stream 1, plus the offset
    (per sample and channel) and perturbation terms when their weights are > 0, in one kernel."""
    ow, pw = float(config.offset_noise_weight), float(config.perturbation_noise_weight)
    if ow > 0 or pw > 0:
        return K.noise_ex(shape, seed=seed, offset=offset, offset_weight=max(ow, 0.0), perturbation_weight=max(pw, 0.0),
                          dtype=dtype, device=device, out=out)
    return K.noise(shape, seed=seed, offset=offset, dtype=dtype, device=device, out=out)


def report_learning_rates(model, lr_scheduler, tensorboard):
    """BaseModelSetup.report_to_tensorboard (modules/modelSetup/BaseModelSetup.py:96-119): the scheduler's
    last lr of each parameter group as `lr/<display name prefix>`, the first group of a prefix winning
    (AdamW's maybe_adjust_lrs is the identity)."""
    lrs = lr_scheduler.get_last_lr()
    names = model.parameters.display_name_mapping()
    if len(lrs) != len(names):
        raise ValueError(f"{len(lrs)} learning rates for {len(names)} parameter groups")
    reported = {}
    for lr, name in zip(lrs, names):
        reported.setdefault(name.split("/")[0], lr)
    for name, lr in reported.items():
        tensorboard.add_scalar(f"lr/{name}", lr, model.train_progress.global_step)


def nhwc_pair(data: dict, C: int):
    """(pred NHWC bf16 [B,h,w,cpad], target NHWC [B,h,w,C]) for the loss kernel: the private kernel
    tensors predict() returned, or -- when a caller hands [B,C,h,w] tensors of its own -- their
    NHWC restatement (pred padded to 8 channels, the kernel's 16-byte row granule)."""
    if "_predicted_nhwc" in data:
        return data["_predicted_nhwc"], data["_target_nhwc"]
    p, t = data["predicted"], data["target"]
    if p.dim() == 4 and p.shape[1] == C and p.shape[-1] != C:
        p = p.permute(0, 2, 3, 1)
        t = t.permute(0, 2, 3, 1)
    cpad = (p.shape[-1] + 7) // 8 * 8
    if cpad != p.shape[-1]:
        p = torch.nn.functional.pad(p, (0, cpad - p.shape[-1]))
    return p.to(torch.bfloat16).contiguous(), t.contiguous()


class BaseStableDiffusionXLSetup:
    def __init__(self, train_device, temp_device=None, debug_mode=False, dp_rank=0, dp_world=1):
        self.train_device = torch.device(train_device)
        self.temp_device = temp_device
        self.debug_mode = debug_mode
        self.dp_rank = dp_rank
        self.dp_world = dp_world
        self.graph_inputs = None   # (noise, timestep) drawn outside a captured step (trainer/step_graph.py)

    # ------------------------------------------------------------------------------------------
    @staticmethod
    def _nhwc_latent(lat: torch.Tensor) -> torch.Tensor:
        """batch latent [B, C, h, w] (the reference contract) -> NHWC for the kernels: free when the
        tensor is a channels-last view (this build's loaders), one relayout copy otherwise (mgds)."""
        return lat.permute(0, 2, 3, 1).contiguous()

    def _text(self, model, batch, config, rand, B):
        config = plain(config)
        te1 = batch["text_encoder_1_hidden_state"]
        te2 = batch.get("text_encoder_2_hidden_state")
        pooled = batch.get("text_encoder_2_pooled_state")
        for part, key in ((config.text_encoder, "te1"), (config.text_encoder_2, "te2")):
            p = part.dropout_probability
            if p is not None and p > 0:   # StableDiffusionXLModel.py:266-281 (host mask from Random(seed))
                mask = torch.tensor([rand.random() > p for _ in range(B)], device=te1.device).to(te1.dtype)
                if key == "te1":
                    te1 = te1 * mask[:, None, None]
                else:
                    te2 = te2 * mask[:, None, None]
                    pooled = pooled * mask[:, None]
        ehs, pooled = model.combine_text_encoder_output(te1.to(torch.bfloat16), None if te2 is None else
                                                        te2.to(torch.bfloat16), pooled)
        return ehs, pooled

    def report_to_tensorboard(self, model, config, lr_scheduler, tensorboard):
        report_learning_rates(model, lr_scheduler, tensorboard)

    def graphable(self, config) -> bool:
        """the step has no host-random or host-varying input besides (noise, timestep), so it can be
        captured once and replayed (text dropout draws its mask on the host per step)."""
        config = plain(config)
        parts = [config.text_encoder] + ([config.text_encoder_2] if hasattr(config, "text_encoder_2") else [])
        return all(not (p.dropout_probability or 0) > 0 for p in parts)

    def step_inputs(self, model, batch: dict, config, train_progress, *, deterministic: bool = False, out=None):
        """(noise, timestep) of this micro-step (ModelSetupNoiseMixin._create_noise /
        _get_timestep_discrete): Philox seeded by `batch_seed`, counter = GLOBAL batch index."""
        config = plain(config)
        batch_seed = 0 if deterministic else train_progress.global_step
        lat = batch["latent_image"]
        B = lat.shape[0]
        shape = tuple(self._nhwc_latent(lat).shape) if out is None else tuple(out[0].shape)
        _, h, w, C = shape
        sample0 = self.dp_rank * B                       # global-batch index of this rank's first sample
        noise = draw_noise(config, shape, batch_seed, sample0 * h * w * C, lat.dtype, lat.device,
                           None if out is None else out[0])
        N = model.noise_scheduler.config["num_train_timesteps"]
        if deterministic:
            timestep = torch.full((B,), int(N * 0.5) - 1, dtype=torch.int32, device=lat.device)
            if out is not None:
                timestep = out[1].copy_(timestep)
        else:
            timestep = K.timesteps(B, seed=batch_seed, sample0=sample0, dist=timestep_plan(config), num_train_timesteps=N,
                                   min_s=config.min_noising_strength, max_s=config.max_noising_strength,
                                   shift=config.timestep_shift, bias=config.noising_bias,
                                   weight=config.noising_weight, device=lat.device,
                                   out=None if out is None else out[1])
        return noise, timestep

    def predict(self, model, batch: dict, config, train_progress, *, deterministic: bool = False) -> dict:
        config = plain(config)
        batch_seed = 0 if deterministic else train_progress.global_step
        rand = Random(batch_seed)
        latent = self._nhwc_latent(batch["latent_image"])
        B, h, w, C = latent.shape
        sf = model.vae.config["scaling_factor"]
        ehs, pooled = self._text(model, batch, config, rand, B)
        if self.graph_inputs is not None:
            noise, timestep = self.graph_inputs
        else:
            noise, timestep = self.step_inputs(model, batch, config, train_progress, deterministic=deterministic)
        ptype = model.noise_scheduler.config["prediction_type"]
        unet_in, target, _ = K.ddpm_prologue(latent, noise, timestep, model.noise_scheduler.coeffs, sf,
                                             1 if ptype == "v_prediction" else 0)
        time_ids = None
        if model.unet.cfg.addition_embed:
            time_ids = torch.stack([batch["original_resolution"][0], batch["original_resolution"][1],
                                    batch["crop_offset"][0], batch["crop_offset"][1],
                                    batch["crop_resolution"][0], batch["crop_resolution"][1]], dim=1).to(
                latent.device, torch.float32)
        pred = model.unet(unet_in, timestep, ehs, pooled, time_ids)
        # the reference contract: predicted / target are [B, 4, h, w] (BaseStableDiffusionXLSetup.py:277-291);
        # here they are views of the NHWC kernel tensors (pred carries 4 zero pad channels), which
        # calculate_loss reads directly through the private keys
        return {"loss_type": "target", "timestep": timestep,
                "predicted": pred[..., :C].permute(0, 3, 1, 2), "target": target.permute(0, 3, 1, 2),
                "prediction_type": ptype, "_predicted_nhwc": pred, "_target_nhwc": target}

    def calculate_loss(self, model, batch: dict, data: dict, config) -> torch.Tensor:
        plan = loss_plan(plain(config))
        lw = batch.get("loss_weight")
        lw = lw.to(self.train_device, torch.float32).contiguous() if lw is not None else None
        pred, target = nhwc_pair(data, 4)
        return Fn.MSELossFn.apply(pred, target, lw, data["timestep"], model.noise_scheduler.coeffs, plan["loss_fn"],
                                  plan["gamma"], data.get("prediction_type") == "v_prediction", 1.0,
                                  plan["mse_strength"], float(plan["batch_size_scale"] * plan["ga_scale"]),
                                  1.0 / self.dp_world)
