"""Generate golden fixtures by running the REFERENCE's own code (container only).

    python tests/golden/make_golden.py          # needs /root/reference (read-only)

Imports the reference modules directly (SURVEY.md §8(c) "Directly, with no stubs"):
  modules/modelSetup/mixin/ModelSetupNoiseMixin.py        _create_noise, _get_timestep_discrete/_continuous
  modules/modelSetup/mixin/ModelSetupDiffusionMixin.py    _add_noise_discrete (DDPM)
  modules/modelSetup/mixin/ModelSetupFlowMatchingMixin.py _add_noise_discrete (flow)
  modules/modelSetup/mixin/ModelSetupDiffusionLossMixin.py _diffusion_losses / _flow_matching_losses
  modules/util/optimizer/adamw_extensions.py               patch_adamw (+ bf16_stochastic_rounding)
  modules/util/lr_scheduler_util.py                        lr lambdas
and records inputs + outputs as .npz data.  Nothing of the reference's source is stored.
The fixtures are the pin for oracle/ (tests/test_oracle_golden.py).
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent


def bf16_bits(t: torch.Tensor) -> np.ndarray:
    return t.contiguous().view(torch.int16).numpy().astype(np.uint16)


def main():
    sys.path.insert(0, str(REF))
    from modules.modelSetup.mixin.ModelSetupDiffusionLossMixin import ModelSetupDiffusionLossMixin
    from modules.modelSetup.mixin.ModelSetupDiffusionMixin import ModelSetupDiffusionMixin
    from modules.modelSetup.mixin.ModelSetupFlowMatchingMixin import ModelSetupFlowMatchingMixin
    from modules.modelSetup.mixin.ModelSetupNoiseMixin import ModelSetupNoiseMixin
    from modules.util import lr_scheduler_util as lrs
    from modules.util.config.TrainConfig import TrainConfig
    from modules.util.enum.LossWeight import LossWeight
    from modules.util.enum.TimestepDistribution import TimestepDistribution
    from modules.util.optimizer.adamw_extensions import patch_adamw

    class DiffProbe(ModelSetupNoiseMixin, ModelSetupDiffusionMixin, ModelSetupDiffusionLossMixin):
        pass

    class FlowProbe(ModelSetupNoiseMixin, ModelSetupFlowMatchingMixin, ModelSetupDiffusionLossMixin):
        pass

    cfg = TrainConfig.default_values()
    cfg.train_device = "cpu"
    rec: dict[str, np.ndarray] = {}

    # ---- 1. noise + timesteps, in predict()'s draw order (noise first, same generator) ----------
    for seed in (0, 7):
        for dist, extra in (("UNIFORM", {}), ("LOGIT_NORMAL", {}), ("UNIFORM_SHIFT3", {"timestep_shift": 3.0}),
                            ("LOGIT_NORMAL_B", {"noising_bias": 0.5, "noising_weight": 0.3})):
            c = TrainConfig.default_values()
            c.train_device = "cpu"
            c.timestep_distribution = TimestepDistribution.LOGIT_NORMAL if dist.startswith("LOGIT") \
                else TimestepDistribution.UNIFORM
            for k, v in extra.items():
                setattr(c, k, v)
            p = DiffProbe()
            g = torch.Generator(device="cpu")
            g.manual_seed(seed)
            src = torch.zeros(4, 4, 8, 8)
            noise = p._create_noise(src, c, g)
            t = p._get_timestep_discrete(1000, False, g, 4, c)
            rec[f"noise_{dist}_{seed}"] = noise.numpy()
            rec[f"timestep_{dist}_{seed}"] = t.numpy()
            g2 = torch.Generator(device="cpu")
            g2.manual_seed(seed)
            rec[f"tcont_{dist}_{seed}"] = p._get_timestep_continuous(False, g2, 4, c).numpy()
    p = DiffProbe()
    rec["timestep_deterministic"] = p._get_timestep_discrete(1000, True, torch.Generator().manual_seed(0), 4, cfg).numpy()

    # ---- 1a. offset / perturbation noise terms (_create_noise with the weights > 0), f32 and bf16 sources ----
    for wname, ow, pw in (("off", 0.1, 0.0), ("pert", 0.0, 0.2), ("both", 0.35, 0.05)):
        for dname, dt in (("f32", torch.float32), ("bf16", torch.bfloat16)):
            c = TrainConfig.default_values()
            c.train_device = "cpu"
            c.offset_noise_weight, c.perturbation_noise_weight = ow, pw
            g = torch.Generator(device="cpu").manual_seed(11)
            noise = DiffProbe()._create_noise(torch.zeros(3, 4, 8, 8, dtype=dt), c, g)
            rec[f"noisex_{wname}_{dname}"] = bf16_bits(noise) if dt == torch.bfloat16 else noise.numpy()
            rec[f"noisex_{wname}_w"] = np.array([ow, pw], dtype=np.float64)

    # ---- 1b. timestep transform on recorded draws (feeds the HIP kernel's injected-draw path) ---------
    # the draw the reference makes inside _get_timestep_discrete is re-made from the same seed
    # (torch.rand / torch.normal with the same generator state), then the reference maps it
    n_draw = 512
    for name, dist, extra in (("uniform", "UNIFORM", {}), ("uniform_shift3", "UNIFORM", {"timestep_shift": 3.0}),
                              ("uniform_range", "UNIFORM", {"min_noising_strength": 0.1, "max_noising_strength": 0.9}),
                              ("logitnormal", "LOGIT_NORMAL", {}),
                              ("logitnormal_b", "LOGIT_NORMAL", {"noising_bias": 0.5, "noising_weight": 0.3}),
                              ("logitnormal_shift", "LOGIT_NORMAL", {"timestep_shift": 2.5})):
        c = TrainConfig.default_values()
        c.train_device = "cpu"
        c.timestep_distribution = TimestepDistribution[dist]
        for k, v in extra.items():
            setattr(c, k, v)
        g = torch.Generator(device="cpu").manual_seed(42)
        t = DiffProbe()._get_timestep_discrete(1000, False, g, n_draw, c)
        g = torch.Generator(device="cpu").manual_seed(42)
        if dist == "UNIFORM":
            draws = torch.rand(n_draw, generator=g)
        else:
            draws = torch.normal(c.noising_bias, c.noising_weight + 1.0, size=(n_draw,), generator=g)
        rec[f"tsinj_{name}_draws"] = draws.numpy()
        rec[f"tsinj_{name}_t"] = t.numpy()
        rec[f"tsinj_{name}_cfg"] = np.array([c.min_noising_strength, c.max_noising_strength, c.timestep_shift,
                                             c.noising_bias, c.noising_weight], dtype=np.float64)

    # ---- 2. add noise -------------------------------------------------------------------------------
    torch.manual_seed(123)
    betas = torch.linspace(0.00085 ** 0.5, 0.012 ** 0.5, 1000, dtype=torch.float32) ** 2
    rec["betas"] = betas.numpy()
    x0 = torch.randn(3, 4, 16, 16)
    eps = torch.randn(3, 4, 16, 16)
    t = torch.tensor([0, 517, 999], dtype=torch.int32)
    rec["an_x0"], rec["an_eps"], rec["an_t"] = x0.numpy(), eps.numpy(), t.numpy()
    rec["an_ddpm_f32"] = DiffProbe()._add_noise_discrete(x0, eps, t, betas).numpy()
    rec["an_ddpm_bf16"] = bf16_bits(DiffProbe()._add_noise_discrete(x0.bfloat16(), eps.bfloat16(), t, betas))
    xt, sig = FlowProbe()._add_noise_discrete(x0, eps, t, torch.zeros(1000))
    rec["an_flow_f32"], rec["an_flow_sigma"] = xt.numpy(), sig.numpy()
    xt, _ = FlowProbe()._add_noise_discrete(x0.bfloat16(), eps.bfloat16(), t, torch.zeros(1000))
    rec["an_flow_bf16"] = bf16_bits(xt)

    # ---- 3. losses ------------------------------------------------------------------------------------
    pred = torch.randn(3, 4, 16, 16).bfloat16()
    target = torch.randn(3, 4, 16, 16)
    lw = torch.tensor([1.0, 0.5, 2.0])
    rec["loss_pred"], rec["loss_target"], rec["loss_lw"] = bf16_bits(pred), target.numpy(), lw.numpy()
    for fn in ("CONSTANT", "MIN_SNR_GAMMA", "DEBIASED_ESTIMATION", "P2"):
        for vp in (False, True):
            c = TrainConfig.default_values()
            c.loss_weight_fn = LossWeight[fn]
            data = {"loss_type": "target", "timestep": t.long(), "predicted": pred, "target": target,
                    "prediction_type": "v_prediction" if vp else "epsilon"}
            losses = DiffProbe()._diffusion_losses({"loss_weight": lw}, data, c, torch.device("cpu"), betas=betas)
            rec[f"loss_{fn}_{int(vp)}"] = losses.numpy()
    for fn in ("CONSTANT", "SIGMA"):
        c = TrainConfig.default_values()
        c.loss_weight_fn = LossWeight[fn]
        data = {"loss_type": "target", "timestep": t.long(), "predicted": pred, "target": target}
        rec[f"flowloss_{fn}"] = FlowProbe()._flow_matching_losses({"loss_weight": lw}, data, c, torch.device("cpu"),
                                                                  sigmas=torch.zeros(1000)).numpy()

    # ---- 4. AdamW (+ bf16 stochastic rounding) ---------------------------------------------------------
    torch.manual_seed(5)
    n = 4099
    p0 = (torch.randn(n) * 0.05).bfloat16()
    grads = [(torch.randn(n) * 10 ** (-2 + k)).bfloat16() for k in range(3)]
    rec["adamw_p0"] = bf16_bits(p0)
    for k in range(3):
        rec[f"adamw_g{k}"] = bf16_bits(grads[k])
    for sr in (False, True):
        prm = torch.nn.Parameter(p0.clone())
        opt = torch.optim.AdamW([prm], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, foreach=False,
                                fused=False)
        patch_adamw(opt, sr)
        for k in range(3):
            prm.grad = grads[k].clone()
            torch.manual_seed(1000 + k)  # SR draws come from the global generator
            opt.step()
            st = opt.state[prm]
            rec[f"adamw_sr{int(sr)}_p{k}"] = bf16_bits(prm.data)
            rec[f"adamw_sr{int(sr)}_m{k}"] = bf16_bits(st["exp_avg"])
            rec[f"adamw_sr{int(sr)}_v{k}"] = bf16_bits(st["exp_avg_sq"])
    # fp32 params (LoRA default dtype)
    pf = torch.nn.Parameter(torch.randn(n) * 0.05)
    rec["adamwf_init"] = pf.detach().numpy().copy()
    opt = torch.optim.AdamW([pf], lr=3e-4, weight_decay=1e-2, foreach=False, fused=False)
    patch_adamw(opt, True)
    for k in range(3):
        gk = torch.randn(n) * 10 ** (-2 + k)
        rec[f"adamwf_g{k}"] = gk.numpy()
        pf.grad = gk
        opt.step()
        rec[f"adamwf_p{k}"] = pf.detach().numpy().copy()

    # global clip as GenericTrainer.py:712-713 calls it, on bf16 grads of several tensors
    torch.manual_seed(9)
    gl = [(torch.randn(s) * sc).bfloat16() for s, sc in ((1000, 0.3), (37, 2.0), (4096, 0.05))]
    for i, g in enumerate(gl):
        rec[f"clip_g{i}"] = bf16_bits(g)
    ps = [torch.nn.Parameter(torch.zeros(g.shape, dtype=torch.bfloat16)) for g in gl]
    for prm, g in zip(ps, gl):
        prm.grad = g.clone()
    tot = torch.nn.utils.clip_grad_norm_(ps, 1.0)
    rec["clip_total"] = np.array([tot.float().item()], dtype=np.float32)
    for i, prm in enumerate(ps):
        rec[f"clip_out{i}"] = bf16_bits(prm.grad)

    # ---- 5. LR lambdas ---------------------------------------------------------------------------------
    steps = np.arange(0, 400)
    for name, fn in (("constant", lrs.lr_lambda_warmup(200, lrs.lr_lambda_constant())),
                     ("cosine", lrs.lr_lambda_warmup(50, lrs.lr_lambda_cosine(300))),
                     ("linear", lrs.lr_lambda_warmup(10, lrs.lr_lambda_linear(390)))):
        rec[f"lr_{name}"] = np.array([fn(int(s)) for s in steps], dtype=np.float64)

    np.savez_compressed(OUT / "reference_math.npz", **rec)
    print("wrote", OUT / "reference_math.npz", len(rec), "arrays")


if __name__ == "__main__":
    main()
