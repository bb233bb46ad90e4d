"""Record the reference's loss / timestep / optimizer decisions for enum-typed TrainConfigs
(container only: imports /root/reference read-only, stores data only).

    python tests/golden/make_config_decisions.py   -> tests/golden/config_decisions.json

For the training presets of C1-C5 (training_presets/#sd 1.5.json, #sdxl 1.0.json,
#sdxl 1.0 LoRA.json, #flux LoRA.json) and overrides of every LossScaler / LossWeight /
TimestepDistribution value, the reference's own TrainConfig.from_dict builds the enum-typed
config; the reference's ModelSetupDiffusionLossMixin._diffusion_losses (or _flow_matching_losses
for Flux) is run with it on fixed small tensors and its per-sample losses are recorded next to
the config's field values (as their value strings).  tests/test_config_boundary.py rebuilds an
enum-typed stand-in from those strings and checks the plugin's decisions reproduce the losses.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "config_decisions.json"
PRESETS = {"sd15": "#sd 1.5.json", "sdxl": "#sdxl 1.0.json", "sdxl_lora": "#sdxl 1.0 LoRA.json",
           "flux_lora": "#flux LoRA.json"}
ENUM_FIELDS = ["model_type", "training_method", "loss_scaler", "loss_weight_fn", "timestep_distribution",
               "peft_type", "train_dtype"]
NUM_FIELDS = ["batch_size", "gradient_accumulation_steps", "loss_weight_strength", "mse_strength", "mae_strength",
              "log_cosh_strength", "masked_training", "learning_rate", "min_noising_strength",
              "max_noising_strength", "timestep_shift", "noising_weight", "noising_bias", "lora_rank", "lora_alpha"]


def inputs():
    g = torch.Generator().manual_seed(3)
    pred = torch.randn(4, 4, 8, 8, generator=g).bfloat16()
    target = torch.randn(4, 4, 8, 8, generator=g)
    lw = torch.tensor([1.0, 0.5, 2.0, 1.5])
    t = torch.tensor([0, 250, 517, 999])
    return pred, target, lw, t


def main():
    sys.path.insert(0, str(REF))
    from modules.modelSetup.mixin.ModelSetupDiffusionLossMixin import ModelSetupDiffusionLossMixin
    from modules.util.config.TrainConfig import TrainConfig
    from modules.util.enum.LossScaler import LossScaler
    from modules.util.enum.LossWeight import LossWeight
    from modules.util.enum.TimestepDistribution import TimestepDistribution

    class Probe(ModelSetupDiffusionLossMixin):
        pass

    betas = torch.linspace(0.00085 ** 0.5, 0.012 ** 0.5, 1000, dtype=torch.float32) ** 2
    pred, target, lw, t = inputs()
    cases = []
    for key, fname in PRESETS.items():
        variants = [{}]
        variants += [{"loss_scaler": s, "batch_size": 4, "gradient_accumulation_steps": 3} for s in LossScaler]
        variants += [{"loss_weight_fn": w} for w in LossWeight]
        variants += [{"timestep_distribution": d} for d in (TimestepDistribution.UNIFORM,
                                                             TimestepDistribution.LOGIT_NORMAL)]
        for var in variants:
            c = TrainConfig.default_values()
            with open(REF / "training_presets" / fname) as f:
                c.from_dict(json.load(f))
            for k, v in var.items():
                setattr(c, k, v)
            flow = key.startswith("flux")
            for vp in ((False,) if flow else (False, True)):
                data = {"loss_type": "target", "timestep": t, "predicted": pred, "target": target}
                if not flow:
                    data["prediction_type"] = "v_prediction" if vp else "epsilon"
                    losses = Probe()._diffusion_losses({"loss_weight": lw}, data, c, torch.device("cpu"), betas=betas)
                else:
                    losses = Probe()._flow_matching_losses({"loss_weight": lw}, data, c, torch.device("cpu"),
                                                           sigmas=torch.zeros(1000))
                rec = {"preset": key, "override": {k: str(getattr(v, "value", v)) for k, v in var.items()},
                       "flow": flow, "v_pred": vp,
                       "enum_fields": {k: getattr(c, k).value for k in ENUM_FIELDS},
                       "optimizer": c.optimizer.optimizer.value,
                       "num_fields": {k: getattr(c, k) for k in NUM_FIELDS},
                       "reference_losses": [float(x) for x in losses.tolist()],
                       "reference_loss_mean": float(losses.mean())}
                cases.append(rec)
    with open(OUT, "w") as f:
        json.dump({"inputs": "tests/golden/make_config_decisions.py:inputs()", "cases": cases}, f, indent=1)
    print("wrote", OUT, len(cases), "cases")


if __name__ == "__main__":
    main()
