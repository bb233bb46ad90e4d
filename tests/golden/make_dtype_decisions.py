"""Record the reference's dtype decisions for its own configs (container only: imports /root/reference
read-only, stores data only).

    python tests/golden/make_dtype_decisions.py   -> tests/golden/dtype_decisions.json

For TrainConfig.default_values() and the C1-C5 training presets (plus train / weight / LoRA dtype overrides),
the reference's own TrainConfig resolves the per-part weight dtypes (TrainConfig.weight_dtypes(),
TrainConfig.py:627-647); its dtype_util.create_autocast_context (dtype_util.py:28-49) is called with the list
the setups pass (BaseStableDiffusionXLSetup.py:54-61 / BaseFluxSetup.py:58-65) and enable_grad_scaling
(dtype_util.py:18-20) with parameters of the trainable dtype.  tests/test_dtype_policy.py checks
util/dtype_util.py against these records.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "dtype_decisions.json"
PRESETS = {"sd15": "#sd 1.5.json", "sdxl": "#sdxl 1.0.json", "sdxl_lora": "#sdxl 1.0 LoRA.json",
           "flux_lora": "#flux LoRA.json"}
PARTS = ("unet", "prior", "text_encoder", "text_encoder_2", "vae")


def main():
    sys.path.insert(0, str(REF))
    from modules.util.config.TrainConfig import TrainConfig
    from modules.util.dtype_util import create_autocast_context, enable_grad_scaling
    from modules.util.enum.DataType import DataType
    from modules.util.enum.ModelType import ModelType
    from modules.util.enum.TrainingMethod import TrainingMethod

    variants = [{}, {"train_dtype": DataType.BFLOAT_16}, {"weight_dtype": DataType.BFLOAT_16},
                {"train_dtype": DataType.BFLOAT_16, "weight_dtype": DataType.BFLOAT_16},
                {"train_dtype": DataType.FLOAT_32}, {"lora_weight_dtype": DataType.BFLOAT_16},
                {"training_method": TrainingMethod.LORA}]
    cases = []
    sources = [("default_values", None)] + list(PRESETS.items())
    for key, fname in sources:
        for var in variants:
            c = TrainConfig.default_values()
            if fname:
                with open(REF / "training_presets" / fname) as f:
                    c.from_dict(json.load(f))
            for k, v in var.items():
                setattr(c, k, v)
            wd = c.weight_dtypes()
            flux = c.model_type in (ModelType.FLUX_DEV_1, ModelType.FLUX_FILL_DEV_1)
            lora = c.training_method == TrainingMethod.LORA
            net = wd.prior if flux else wd.unet
            ctx, train_dtype = create_autocast_context(torch.device("cpu"), c.train_dtype, [
                net, wd.text_encoder, wd.text_encoder_2, wd.vae, wd.lora if lora else None, None],
                c.enable_autocast_cache)
            trainable = wd.lora if lora else net
            tdt = trainable.torch_dtype() or torch.float32
            scaler = enable_grad_scaling(c.train_dtype, [torch.nn.Parameter(torch.zeros(1, dtype=tdt))])
            cases.append({
                "source": key, "override": {k: getattr(v, "value", v) for k, v in var.items()},
                "fields": {"model_type": c.model_type.value, "training_method": c.training_method.value,
                           "train_dtype": c.train_dtype.value, "fallback_train_dtype": c.fallback_train_dtype.value,
                           "weight_dtype": c.weight_dtype.value, "lora_weight_dtype": c.lora_weight_dtype.value,
                           "parts": {p: getattr(c, p).weight_dtype.value for p in PARTS}},
                "resolved": {"unet": wd.unet.value, "prior": wd.prior.value, "text_encoder": wd.text_encoder.value,
                             "text_encoder_2": wd.text_encoder_2.value, "vae": wd.vae.value, "lora": wd.lora.value},
                "reference": {"compute": train_dtype.value, "autocast": bool(getattr(ctx, "_enabled", False)),
                              "grad_scaler": bool(scaler)},
            })
    with open(OUT, "w") as f:
        json.dump({"cases": cases}, f, indent=1)
    print("wrote", OUT, len(cases), "cases")


if __name__ == "__main__":
    main()
